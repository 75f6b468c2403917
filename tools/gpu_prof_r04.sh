#!/bin/bash
# Round-4 record: rocprofv3 kernel trace + stats of the default bench on the final tree, the
# roofline kernel's cold launches from that trace against bench.py's own figure, the per-kernel
# cycle breakdown, and the PMC traffic passes of the roofline kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
  -- python3 bench.py > gpurun_out/r04/bench_prof.log 2>&1 || { echo "rocprof bench failed rc=$?"; tail -5 gpurun_out/r04/bench_prof.log; exit 1; }
grep '^{' gpurun_out/r04/bench_prof.log > gpurun_out/r04/bench_under_rocprof.json
cut -c1-300 gpurun_out/r04/bench_under_rocprof.json
T=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
python3 tools/rocprof_roofline.py "$T" gpurun_out/r04/bench_under_rocprof.json \
  gpurun_out/r04/rocprof_roofline_kernel_stats.csv | tee gpurun_out/r04/rocprof_roofline.txt
python3 tools/cycle_trace.py "$T" 15 k_rowpa > gpurun_out/r04/cycle_trace.txt 2>&1
rm -f "$T"
tail -1 gpurun_out/r04/cycle_trace.txt
for f in $(find gpurun_out/prof -name "*stats.csv"); do cp "$f" gpurun_out/r04/rocprof_$(basename "$f"); done
if [ "${PMC:-1}" = "1" ]; then
  timeout -k 10 600 python3 tools/pmc_traffic.py r04 rowpat > gpurun_out/r04/pmc_rowpat.log 2>&1 || { echo "pmc failed rc=$?"; tail -5 gpurun_out/r04/pmc_rowpat.log; exit 1; }
  tail -3 gpurun_out/r04/pmc_rowpat.log
fi
if [ "${PMC_AB:-0}" = "1" ]; then
  # the uniform stencil kernel against the general row-pair kernel, with L2 hit / miss counts
  PMC_L2=1 PMC_TAG=_uni timeout -k 10 300 python3 tools/pmc_traffic.py r04 rowpat > gpurun_out/r04/pmc_uni_l2.log 2>&1 || { echo "pmc uni failed rc=$?"; tail -5 gpurun_out/r04/pmc_uni_l2.log; exit 1; }
  MLAMG_RP_UNI=0 PMC_L2=1 PMC_TAG=_pair timeout -k 10 300 python3 tools/pmc_traffic.py r04 rowpat > gpurun_out/r04/pmc_pair_l2.log 2>&1 || { echo "pmc pair failed rc=$?"; tail -5 gpurun_out/r04/pmc_pair_l2.log; exit 1; }
  grep -h -E 'traffic_over|TCC_|driver' gpurun_out/r04/pmc_uni_l2.log gpurun_out/r04/pmc_pair_l2.log
fi
