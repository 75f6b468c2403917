#!/bin/bash
# Round-3 record on the final tree: rocprofv3 kernel-trace summary of the default bench, the
# per-kernel cycle breakdown from that trace, and the PMC traffic passes of the roofline kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
  -- python3 bench.py > gpurun_out/bench_prof.log 2>&1 || { echo "rocprof bench failed rc=$?"; tail -5 gpurun_out/bench_prof.log; exit 1; }
grep '^{' gpurun_out/bench_prof.log | cut -c1-300
T=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
python3 tools/cycle_trace.py "$T" 15 > gpurun_out/cycle_trace_final.txt 2>&1
rm -f "$T"
tail -1 gpurun_out/cycle_trace_final.txt
timeout -k 10 600 python3 tools/pmc_traffic.py r03 rowpat > gpurun_out/pmc_rowpat.log 2>&1 || { echo "pmc failed rc=$?"; tail -5 gpurun_out/pmc_rowpat.log; exit 1; }
tail -3 gpurun_out/pmc_rowpat.log
find gpurun_out/prof -name "*stats.csv"
