#!/bin/bash
# Round 4: every BASELINE config's cycle rate on the current tree (profiles/r04/configs.json) and
# the C2 cycle's per-kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/bench_configs.py --steps 50 --cpu-cycles 3 --out gpurun_out/r04/configs.json > gpurun_out/r04/configs.log 2>&1 || { echo "configs failed rc=$?"; tail -5 gpurun_out/r04/configs.log; exit 1; }
rm -rf gpurun_out/prof_c2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_c2 -o c2 -- python3 tools/cycle_run.py C2 40 > gpurun_out/r04/cycle_run_c2.log 2>&1 || { echo "c2 trace failed rc=$?"; tail -5 gpurun_out/r04/cycle_run_c2.log; exit 1; }
T=$(find gpurun_out/prof_c2 -name "*kernel_trace.csv" | head -1)
python3 tools/cycle_trace.py "$T" 15 > gpurun_out/r04/cycle_trace_c2.txt 2>&1
rm -rf gpurun_out/prof_c2
tail -2 gpurun_out/r04/cycle_trace_c2.txt
# the multi-GPU compute floor (timing-only communicator) on this tree, world 1/2/4/8, with the
# default and a deeper partition
timeout -k 10 600 python3 tools/dist_rank_timing.py --worlds 1,2,4,8 --steps 40 --min-rows 50000,5000 > gpurun_out/r04/dist_rank_timing.log 2>&1 || { echo "dist timing failed rc=$?"; tail -5 gpurun_out/r04/dist_rank_timing.log; exit 1; }
tail -3 gpurun_out/r04/dist_rank_timing.log
