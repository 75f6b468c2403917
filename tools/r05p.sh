#!/bin/bash
# A/B of sorted-kernel build knobs on the C4 bench (alternating, 2 rounds)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05p; mkdir -p $O
val() { grep '^{' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
B="python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-c3 --no-varcoef"
for i in 1 2 3; do
  for v in default chain8 c8w6 chain4 wav6; do
    if [ $v = default ]; then L=ml-amg_amd/mlamg/libmlamg_hip.so; else L=tools/abx/libmlamg_$v.so; fi
    MLAMG_LIB=$L timeout -k 10 300 $B > $O/b_$v.log 2>&1 || exit 1; echo "$v $(val $O/b_$v.log)"
  done
done
