#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05k; mkdir -p $O
export TMPDIR=/tmp
for f in 0 1; do
  rm -rf gpurun_out/prof_cfg
  MLAMG_FACTORED_P0=$f timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_cfg -o t -- python3 tools/cycle_run.py C4 40 > $O/cycle_run_f$f.log 2>&1 || { echo "trace failed"; exit 1; }
  T=$(find gpurun_out/prof_cfg -name "*kernel_trace.csv" | head -1)
  python3 tools/cycle_trace.py "$T" 15 > $O/cycle_trace_f$f.txt 2>&1
  rm -rf gpurun_out/prof_cfg
  echo f$f; tail -1 $O/cycle_trace_f$f.txt
done
