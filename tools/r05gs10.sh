set -o pipefail
O=gpurun_out/r05gs10; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pyamg_sa.py > $O/pytest.log 2>&1 && \
timeout -k 10 600 python -u tools/pyamg_sa_bench.py --case poisson3d:128 --case poisson2d:1024 --out $O/on.json > $O/on.log 2>&1 && \
true
