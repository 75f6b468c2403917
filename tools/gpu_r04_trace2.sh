#!/bin/bash
# Traced C4 cycle with the default library and with variant $V (timing only), side by side.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
for lib in default $V; do
  rm -rf gpurun_out/prof_t2
  if [ $lib = default ]; then unset MLAMG_LIB; else export MLAMG_LIB=$PWD/tools/abv/libmlamg_$V.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_t2 -o c4 -- python3 tools/cycle_run.py C4 30 > gpurun_out/r04/t2_run_$lib.log 2>&1 || { echo "trace failed"; exit 1; }
  T=$(find gpurun_out/prof_t2 -name "*kernel_trace.csv" | head -1)
  python3 tools/cycle_trace.py "$T" 15 k_rowpa > gpurun_out/r04/t2_trace_$lib.txt 2>&1
  rm -rf gpurun_out/prof_t2
done
paste -d'|' <(cut -c1-16 gpurun_out/r04/t2_trace_default.txt) <(cut -c1-120 gpurun_out/r04/t2_trace_$V.txt)
