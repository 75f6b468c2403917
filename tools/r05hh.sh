set -o pipefail
O=gpurun_out/r05hh; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pyamg_sa.py > $O/pytest_sa.log 2>&1 && \
timeout -k 10 600 python -u tools/gmres_orthog_bench.py --out $O/gmres_orthog.json > $O/gmres_orthog.log 2>&1
