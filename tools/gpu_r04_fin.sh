#!/bin/bash
# Fused norm finalize: parity tests, then the C4 and C2 cycle with and without it (same box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hierarchy.py tests/test_gpu_distributed_loopback.py tests/test_gpu_configs.py > gpurun_out/r04/fin_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/r04/fin_tests.log; exit 1; }
tail -2 gpurun_out/r04/fin_tests.log
val() { grep '^{' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
B="python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-c3 --no-varcoef"
for i in 1 2; do
  timeout -k 10 300 $B > gpurun_out/r04/fn_a.log 2>&1 || exit 1; echo "fused C4 $(val gpurun_out/r04/fn_a.log)"
  MLAMG_FUSED_NORM=0 timeout -k 10 300 $B > gpurun_out/r04/fn_b.log 2>&1 || exit 1; echo "separate C4 $(val gpurun_out/r04/fn_b.log)"
done
for i in 1 2; do
  timeout -k 10 200 python3 tools/cycle_run.py C2 200 > gpurun_out/r04/fn_c2a.log 2>&1 || exit 1; echo "fused C2 $(tail -1 gpurun_out/r04/fn_c2a.log)"
  MLAMG_FUSED_NORM=0 timeout -k 10 200 python3 tools/cycle_run.py C2 200 > gpurun_out/r04/fn_c2b.log 2>&1 || exit 1; echo "separate C2 $(tail -1 gpurun_out/r04/fn_c2b.log)"
done
