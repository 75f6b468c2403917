# ad-hoc GPU session (edited per experiment)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python tools/bench_configs.py --out gpurun_out/configs.json > gpurun_out/configs.log 2>&1 || { tail -20 gpurun_out/configs.log; exit 1; }
tail -6 gpurun_out/configs.log | cut -c1-300
