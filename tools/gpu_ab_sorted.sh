#!/bin/bash
# A/B of library variants on one box (${VARDIR:-tools/variants}/lib_<name>.so; "new" = the in-tree build):
# the coarse-operator kernel table and a short bench run each, twice, in alternation.
#   bash tools/gpu_ab_sorted.sh base new [other variants...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
for v in "$@"; do
  if [ $v = new ]; then unset MLAMG_LIB; else export MLAMG_LIB=$PWD/${VARDIR:-tools/variants}/lib_$v.so; fi
  timeout -k 10 300 python -u tools/coarse_formats.py 216 --levels 0 1 2 3 --out gpurun_out/cf_$v.json > gpurun_out/cf_$v.log 2>&1 || { echo "cf $v failed"; tail -5 gpurun_out/cf_$v.log; exit 1; }
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-c3 --no-varcoef --steps 50 > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/bench_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
done
