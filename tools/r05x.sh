set -o pipefail
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_hierarchy.py tests/test_gpu_configs.py tests/test_gpu_distributed_loopback.py > $O/pytest.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err
