#!/bin/bash
# A/B of library builds on one box: a short bench per build, twice, in alternation
# ("new" = the in-tree build, otherwise ${VARDIR:-tools/ab}/lib_<name>.so).
#   bash tools/ab_lib.sh new w6
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    if [ $v = new ]; then unset MLAMG_LIB; else export MLAMG_LIB=$PWD/${VARDIR:-tools/ab}/lib_$v.so; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-c3 --no-varcoef --steps 50 > gpurun_out/ablib_$v.json 2> gpurun_out/ablib_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/ablib_$v.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ablib_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
  done
done
