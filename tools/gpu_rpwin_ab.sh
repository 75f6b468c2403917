#!/bin/bash
# rowpat LDS window: parity tests, then same-box bench A/B (window off / on at workgroup sizes)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hierarchy.py -k "rowpat or vector_format or multilevel_setup" > gpurun_out/t_rpwin.log 2>&1 || { tail -30 gpurun_out/t_rpwin.log; exit 1; }
tail -2 gpurun_out/t_rpwin.log
val() { grep '^{' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_us"])'; }
for v in ${RPWIN_VARIANTS:-0 256 512 1024 0}; do
  if [ $v = 0 ]; then export MLAMG_RP_WIN=0; else export MLAMG_RP_WIN=1; fi
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-c3 --no-varcoef > gpurun_out/ab_rpwin_$v.log 2>&1 || { tail -20 gpurun_out/ab_rpwin_$v.log; exit 1; }
  echo "win=$v $(val gpurun_out/ab_rpwin_$v.log)"
done
