#!/bin/bash
# A/B: sorted kernel long-row instantiation threshold (48 default vs 32 vs 3), C4 bench + trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05o; mkdir -p $O
export TMPDIR=/tmp
val() { grep '^{' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
B="python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-c3 --no-varcoef"
for i in 1 2; do
  for v in default lr32 lr3; do
    if [ $v = default ]; then L=ml-amg_amd/mlamg/libmlamg_hip.so; else L=tools/abx/libmlamg_$v.so; fi
    MLAMG_LIB=$L timeout -k 10 300 $B > $O/b_$v.log 2>&1 || exit 1; echo "$v $(val $O/b_$v.log)"
  done
done
for v in lr32; do
  rm -rf gpurun_out/prof_cfg
  MLAMG_LIB=tools/abx/libmlamg_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_cfg -o t -- python3 tools/cycle_run.py C4 40 > $O/cr_$v.log 2>&1 || exit 1
  T=$(find gpurun_out/prof_cfg -name "*kernel_trace.csv" | head -1)
  python3 tools/cycle_trace.py "$T" 15 > $O/trace_$v.txt 2>&1
  rm -rf gpurun_out/prof_cfg
done
