#!/bin/bash
# k_rowpat_uni with the epilogue operands prefetched a chunk ahead (MLAMG_UNI_EPF build) against
# the default: C4 bench, alternating on one box, then one traced cycle of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
V=${V:-epf}
val() { grep '^{' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
B="python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-c3 --no-varcoef"
for i in 1 2 3; do
  timeout -k 10 300 $B > gpurun_out/r04/ep_a.log 2>&1 || exit 1; echo "default $(val gpurun_out/r04/ep_a.log)"
  MLAMG_LIB=$PWD/tools/abv/libmlamg_$V.so timeout -k 10 300 $B > gpurun_out/r04/ep_b.log 2>&1 || exit 1; echo "$V $(val gpurun_out/r04/ep_b.log)"
done
for lib in default $V; do
  rm -rf gpurun_out/prof_ep
  if [ $lib = default ]; then unset MLAMG_LIB; else export MLAMG_LIB=$PWD/tools/abv/libmlamg_$V.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_ep -o c4 -- python3 tools/cycle_run.py C4 30 > gpurun_out/r04/ep_run_$lib.log 2>&1 || { echo "trace failed"; exit 1; }
  T=$(find gpurun_out/prof_ep -name "*kernel_trace.csv" | head -1)
  python3 tools/cycle_trace.py "$T" 15 k_rowpa > gpurun_out/r04/ep_trace_$lib.txt 2>&1
  rm -rf gpurun_out/prof_ep
  echo "$lib"; grep -E "rowpat|cycles" gpurun_out/r04/ep_trace_$lib.txt
done
