# ad-hoc GPU session (edited per experiment)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/kernel_roofline.py > gpurun_out/kr_a.md 2>/dev/null || exit 1
MLAMG_LIB=$PWD/tools/variants/libmlamg_srt256.so timeout -k 10 300 python tools/kernel_roofline.py > gpurun_out/kr_b.md 2>/dev/null || exit 1
paste -d'|' <(cut -d'|' -f2,3,4,8 gpurun_out/kr_a.md) <(cut -d'|' -f4,8 gpurun_out/kr_b.md)
