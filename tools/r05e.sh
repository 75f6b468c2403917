#!/bin/bash
# Per-kernel cycle traces (C4, C2) of the round-5 tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05e; mkdir -p $O
export TMPDIR=/tmp
for c in C4 C2; do
  rm -rf gpurun_out/prof_cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_cfg -o t -- python3 tools/cycle_run.py $c 40 > $O/cycle_run_$c.log 2>&1 || { echo "trace $c failed"; exit 1; }
  T=$(find gpurun_out/prof_cfg -name "*kernel_trace.csv" | head -1)
  python3 tools/cycle_trace.py "$T" 15 > $O/cycle_trace_$c.txt 2>&1
  rm -rf gpurun_out/prof_cfg
  echo $c; tail -1 $O/cycle_trace_$c.txt
done
