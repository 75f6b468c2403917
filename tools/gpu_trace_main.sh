#!/bin/bash
# per-kernel breakdown of the main C4 bench cycle (no C3 / variable-coefficient legs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/tr_main
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_main -o b -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-c3 --no-varcoef > gpurun_out/tr_main.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/tr_main.log; exit 1; }
python3 tools/cycle_trace.py gpurun_out/tr_main/b_kernel_trace.csv 15 > gpurun_out/cycle_trace_main.txt 2>&1
rm -f gpurun_out/tr_main/b_kernel_trace.csv
cat gpurun_out/cycle_trace_main.txt
