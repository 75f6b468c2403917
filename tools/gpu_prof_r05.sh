#!/bin/bash
# Round-5 record: rocprofv3 kernel trace + stats of the default bench on the final tree, the
# roofline kernel's cold launches from that trace against bench.py's own figure, the per-kernel
# cycle breakdown, and the PMC traffic passes of the roofline kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r05prof}
mkdir -p $OUT
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
  -- python3 bench.py > $OUT/bench_prof.log 2>&1 || { echo "rocprof bench failed rc=$?"; tail -5 $OUT/bench_prof.log; exit 1; }
grep '^{' $OUT/bench_prof.log > $OUT/bench_under_rocprof.json
cut -c1-300 $OUT/bench_under_rocprof.json
T=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
python3 tools/rocprof_roofline.py "$T" $OUT/bench_under_rocprof.json \
  $OUT/rocprof_roofline_kernel_stats.csv | tee $OUT/rocprof_roofline.txt
python3 tools/cycle_trace.py "$T" 15 k_rowpa > $OUT/cycle_trace.txt 2>&1
rm -f "$T"
tail -1 $OUT/cycle_trace.txt
for f in $(find gpurun_out/prof -name "*stats.csv"); do cp "$f" $OUT/rocprof_$(basename "$f"); done
if [ "${PMC:-1}" = "1" ]; then
  timeout -k 10 600 python3 tools/pmc_traffic.py r05 rowpat > $OUT/pmc_rowpat.log 2>&1 || { echo "pmc failed rc=$?"; tail -5 $OUT/pmc_rowpat.log; exit 1; }
  tail -3 $OUT/pmc_rowpat.log
fi
