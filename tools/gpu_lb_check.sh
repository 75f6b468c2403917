set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
MLAMG_DEVICE_CACHE_MB=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_distributed_loopback.py -k c4_world8 > gpurun_out/lb_nocache.log 2>&1; echo "nocache rc=$?"; tail -1 gpurun_out/lb_nocache.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_distributed_loopback.py -k c4_world8 > gpurun_out/lb_cache.log 2>&1; echo "cache rc=$?"; tail -1 gpurun_out/lb_cache.log
