#!/bin/bash
# The one GPU job runner (replaces the per-run job scripts of rounds 1-5).
#
#   bash tools/gpujob.sh TAG STEP [STEP ...]
#
# STEP is "name:seconds:command" (the command is run by bash; its stdout and stderr go to
# gpurun_out/TAG/name.log), or one of the presets
#   suite       the GPU parity suite (pytest -m gpu, per-test thread timeouts)
#   smoke       __graft_entry__.smoke()
#   bench       the default bench line (gpurun_out/TAG/bench.json)
#   prof        rocprofv3 --kernel-trace --stats of a short bench (gpurun_out/TAG/prof)
#   pytest=ARGS pytest -m gpu on ARGS (a file or node id), e.g. pytest=tests/test_gpu_configs.py
#
# Each step runs under its own `timeout -k 10`; the first step that fails ends the job, so a GPU
# fault, abort, segfault or time limit is never followed by more GPU work.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
PYT="python -u -m pytest -x -q -rf --timeout 300 --timeout-method thread -m gpu"
for step in "$@"; do
  case "$step" in
    suite) step="suite:900:$PYT tests" ;;
    smoke) step="smoke:300:python __graft_entry__.py smoke" ;;
    bench) step="bench:600:python bench.py > $OUT/bench.json" ;;
    prof) step="prof:600:rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o p -- python bench.py --steps 20 --no-cpu-baseline > $OUT/prof_bench.json" ;;
    pytest=*) step="pytest_$(basename "${step#pytest=}" .py | tr -c 'A-Za-z0-9_\n' _):900:$PYT ${step#pytest=}" ;;
  esac
  name=${step%%:*}
  rest=${step#*:}
  secs=${rest%%:*}
  cmd=${rest#*:}
  t0=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s"
  tail -4 "$OUT/$name.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
