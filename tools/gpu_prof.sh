#!/bin/bash
# rocprofv3 kernel-trace summary of the default bench command + the PMC traffic passes of the
# roofline kernel. Each GPU step has its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof
echo "=== rocprof bench"; date
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
  -- python bench.py > gpurun_out/bench_prof.log 2>&1 || { echo "rocprof bench failed rc=$?"; tail -5 gpurun_out/bench_prof.log; exit 1; }
tail -1 gpurun_out/bench_prof.log | cut -c1-600
echo "=== pmc rowpat"; date
timeout -k 10 600 python tools/pmc_traffic.py ${ROUND:-r01} rowpat > gpurun_out/pmc_rowpat.log 2>&1 || { echo "pmc failed rc=$?"; tail -5 gpurun_out/pmc_rowpat.log; exit 1; }
tail -3 gpurun_out/pmc_rowpat.log
find gpurun_out/prof -name "*kernel_stats.csv" | head
