# ad-hoc GPU session (edited per experiment)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || { tail -20 gpurun_out/bench_prof.log; exit 1; }
grep '"value"' gpurun_out/bench_prof.log | cut -c1-300
