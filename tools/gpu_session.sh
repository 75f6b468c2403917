# ad-hoc GPU session (edited per experiment)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/kernel_roofline.py > gpurun_out/kernel_roofline.md 2> gpurun_out/kernel_roofline.err || { tail -20 gpurun_out/kernel_roofline.err; exit 1; }
cat gpurun_out/kernel_roofline.md
