#!/bin/bash
# One GPU session: parity tests, smoke, a small and a full bench. Each GPU step has its own
# time limit; a crash/timeout (rc > 1) ends the script before any further GPU work.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name" ; date
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" >> "$OUT/$name.log"
  echo "$name rc=$rc"
  tail -5 "$OUT/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step pytest_gpu 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -rf
fi
if [ "$MODE" = all ] || [ "$MODE" = smoke ]; then
  step smoke 300 python __graft_entry__.py smoke
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench_small 600 python bench.py --n 64 --steps 20 --warmup 3 --no-cpu-baseline --verbose
  step bench_full 900 python bench.py --verbose
fi
if [ "$MODE" = prof ]; then
  rm -rf $OUT/prof
  step rocprof_bench 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python bench.py --steps 30 --warmup 3 --no-cpu-baseline
  export MLAMG_FMT=sell_dict
  step rocprof_spmv 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o spmv -- python tools/spmv_driver.py
  unset MLAMG_FMT
  step pmc_dict 600 python tools/pmc_traffic.py ${ROUND:-r01} sell_dict
  step pmc_sell 600 python tools/pmc_traffic.py ${ROUND:-r01} sell
  step pmc_sorted 600 python tools/pmc_traffic.py ${ROUND:-r01} sorted
fi
if [ "$MODE" = dist ]; then
  step bench_dist1 900 python bench.py --dist --steps 30 --warmup 3
fi
