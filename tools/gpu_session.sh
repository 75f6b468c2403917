# ad-hoc GPU session (edited per experiment)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_hierarchy.py tests/test_gpu_distributed.py -q -m gpu --timeout 120 --timeout-method thread -x > gpurun_out/pt5.log 2>&1 || { tail -30 gpurun_out/pt5.log; exit 1; }
tail -1 gpurun_out/pt5.log
timeout -k 10 120 python tools/rowpat_ops.py || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_k.log 2>&1 || { tail -20 gpurun_out/bench_k.log; exit 1; }
grep -o '"value": [0-9.]*\|"avg_launch_us": [0-9.]*\|"frac": [0-9.]*' gpurun_out/bench_k.log
