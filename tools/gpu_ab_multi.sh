#!/bin/bash
# Same-box A/B of the in-tree library against variants (tools/abx/lib_<name>.so), C4 bench
# (no C3 / variable-coefficient legs), alternating, R rounds.  bash tools/gpu_ab_multi.sh R v1 v2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=$1; shift
val() { grep '^{' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for i in $(seq "$R"); do
  for v in base "$@"; do
    if [ $v = base ]; then unset MLAMG_LIB; else export MLAMG_LIB=$PWD/tools/abx/lib_$v.so; fi
    timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-c3 --no-varcoef > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
    echo "$v $(val gpurun_out/ab_$v.log)"
  done
done
