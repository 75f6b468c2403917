set -o pipefail
O=gpurun_out/r05s; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_distributed.py tests/test_gpu_distributed_loopback.py > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --dist --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_dist1.json 2> $O/bench_dist1.err
