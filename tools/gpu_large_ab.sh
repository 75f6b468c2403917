# two-level amg_2_v beyond the fused engine: device allocation cache off vs on (same box).
# Each GPU step has its own time limit; a failure ends the script.
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
MLAMG_DEVICE_CACHE_MB=0 timeout -k 10 400 python -u tools/amg2v_large.py 320 512 1024 > gpurun_out/large_nocache.log 2>&1 || { echo fail1; tail -20 gpurun_out/large_nocache.log; exit 1; }
grep grid gpurun_out/large_nocache.log
timeout -k 10 400 python -u tools/amg2v_large.py 320 512 1024 > gpurun_out/large_cache.log 2>&1 || { echo fail2; tail -20 gpurun_out/large_cache.log; exit 1; }
grep grid gpurun_out/large_cache.log
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_device_cache.py tests/test_gpu_coarse_pcg.py > gpurun_out/cache_tests2.log 2>&1 || { tail -20 gpurun_out/cache_tests2.log; exit 1; }
tail -1 gpurun_out/cache_tests2.log
