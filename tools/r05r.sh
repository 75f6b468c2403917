set -o pipefail
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_distributed.py > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --dist --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_dist1.json 2> $O/bench_dist1.err
