#!/bin/bash
# A/B of runtime knobs on one box: a short bench per setting, twice, in alternation.
#   bash tools/ab_env.sh "" "MLAMG_NO_CACHED_LOADS=1" ...   ("" = defaults)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-c3 --no-varcoef --steps 50 > gpurun_out/abenv_$i.json 2> gpurun_out/abenv_$i.err || { echo "bench [$v] failed"; tail -5 gpurun_out/abenv_$i.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/abenv_$i.json').read().strip().splitlines()[-1]); print('[$v]', d['value'], d['ms_per_step'])"
  done
done
