# loopback executor tests (world 2..8 on one GPU) after the device allocation cache; each GPU
# step has its own time limit; a failure ends the script.
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_distributed_loopback.py tests/test_gpu_device_cache.py -rf > gpurun_out/lb_cache.log 2>&1; rc=$?
tail -3 gpurun_out/lb_cache.log; exit $rc
