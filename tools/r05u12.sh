set -o pipefail
O=gpurun_out/r05u12; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pyamg_sa.py -k "gauss_seidel" > $O/pytest.log 2>&1 && \
timeout -k 10 600 python -u tools/pyamg_sa_bench.py --case poisson2d:1024 --out $O/p.json > $O/p.log 2>&1 && \
timeout -k 10 600 python -u tools/amg2v_large.py 1024 > $O/a.jsonl 2> $O/err.log
