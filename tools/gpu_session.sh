# ad-hoc GPU session (edited per experiment)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/profA gpurun_out/profB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profA -o a -- python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/benchA.log 2>&1 || exit 1
MLAMG_LIB=$PWD/tools/variants/libmlamg_vu8.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profB -o b -- python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/benchB.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/benchA.log gpurun_out/benchB.log
