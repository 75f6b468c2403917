set -o pipefail
O=gpurun_out/r05gs8; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof3d -o run -- python3 tools/pyamg_sa_trace.py poisson3d:128 3 > $O/trace3d.log 2>&1 ; 
find $O -name "*kernel_trace.csv" -delete; find $O -name "*.db" -delete; du -sh $O
