#!/bin/bash
# Same-box A/B of the default library against a variant (MLAMG_LIB), C4 bench, alternating runs.
#   bash tools/ab_variant.sh tools/variants/libmlamg_<x>.so [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$1
N=${2:-2}
EXTRA=${AB_EXTRA:-}
val() { grep '^{' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for i in $(seq "$N"); do
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-c3 --no-varcoef > gpurun_out/ab_a.log 2>&1 || exit 1
  echo "default $(val gpurun_out/ab_a.log)"
  MLAMG_LIB=$PWD/$V timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-c3 --no-varcoef > gpurun_out/ab_b.log 2>&1 || exit 1
  echo "variant $(val gpurun_out/ab_b.log)"
done
