set -o pipefail
O=gpurun_out/r05lpr; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in 8 16; do
  MLAMG_GS_WAVE_LPR=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$L -o run -- python3 tools/pyamg_sa_trace.py poisson2d:1024 3 > $O/t$L.log 2>&1 || exit 1
  MLAMG_GS_WAVE_LPR=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/q$L -o run -- python3 tools/pyamg_sa_trace.py poisson3d:64 5 > $O/u$L.log 2>&1 || exit 1
done
find $O -name "*kernel_trace.csv" -delete; find $O -name "*.db" -delete
