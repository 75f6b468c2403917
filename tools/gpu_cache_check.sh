# device allocation cache: its GPU tests + PCG tests, then the 320^2 / 512^2 setup / cycle / free
# split. Each GPU step has its own time limit; a failure ends the script.
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp


MLAMG_TIMING=1 timeout -k 10 300 python -u tools/amg2v_large_phases.py 320 > gpurun_out/cache_phases.log 2>&1 || { echo ph-fail; tail -20 gpurun_out/cache_phases.log; exit 1; }
grep grid gpurun_out/cache_phases.log | cut -c1-20,330-900
timeout -k 10 300 python -u tools/amg2v_large.py 320 > gpurun_out/cache_large.log 2>&1 || { echo large-fail; tail -20 gpurun_out/cache_large.log; exit 1; }
grep grid gpurun_out/cache_large.log
