# ad-hoc GPU session (edited per experiment)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/pmc_traffic.py r01 rowpat > gpurun_out/pmc_rowpat.log 2>&1 || { tail -20 gpurun_out/pmc_rowpat.log; exit 1; }
cat gpurun_out/pmc/spmv_c4_pmc_rowpat.json
