#!/bin/bash
# An environment-variable variant ($ENVV, e.g. MLAMG_SRT_UG=1): its parity tests (pytest -k $K),
# then the C4 bench alternating with the default, then one traced cycle of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
env $ENVV timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hierarchy.py tests/test_gpu_kernels.py tests/test_gpu_partition_formats.py -k "${K:-sorted or exact or c4_full or results_do_not or partition or local}" > gpurun_out/r04/env_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/r04/env_tests.log; exit 1; }
tail -1 gpurun_out/r04/env_tests.log
val() { grep '^{' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["setup_s"]["total"] if isinstance(d.get("setup_s"), dict) else d.get("setup_s"))'; }
B="python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-c3 --no-varcoef"
for i in 1 2 3; do
  timeout -k 10 300 $B > gpurun_out/r04/ev_a.log 2>&1 || exit 1; echo "default $(val gpurun_out/r04/ev_a.log)"
  env $ENVV timeout -k 10 300 $B > gpurun_out/r04/ev_b.log 2>&1 || exit 1; echo "$ENVV $(val gpurun_out/r04/ev_b.log)"
done
for v in default variant; do
  rm -rf gpurun_out/prof_ev
  if [ $v = default ]; then E=""; else E="$ENVV"; fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_ev -o c4 -- python3 tools/cycle_run.py C4 30 > gpurun_out/r04/ev_run_$v.log 2>&1 || { echo "trace failed"; exit 1; }
  T=$(find gpurun_out/prof_ev -name "*kernel_trace.csv" | head -1)
  python3 tools/cycle_trace.py "$T" 15 k_rowpa > gpurun_out/r04/ev_trace_$v.txt 2>&1
  rm -rf gpurun_out/prof_ev
done
paste -d'|' <(cut -c1-16 gpurun_out/r04/ev_trace_default.txt) <(cut -c1-110 gpurun_out/r04/ev_trace_variant.txt)
