#!/bin/bash
# Paired kernel traces of the bench on one box, one per library build ("new" = the in-tree
# build, otherwise ${VARDIR:-tools/abx}/lib_<name>.so), summarised per kernel of one cycle.
#   bash tools/trace_ab.sh base new
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for v in "$@"; do
  if [ $v = new ]; then unset MLAMG_LIB; else export MLAMG_LIB=$PWD/${VARDIR:-tools/abx}/lib_$v.so; fi
  rm -rf gpurun_out/tr_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_$v -o b -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 --no-varcoef > gpurun_out/tr_$v.log 2>&1 || { echo "trace $v failed"; tail -5 gpurun_out/tr_$v.log; exit 1; }
  python tools/cycle_trace.py gpurun_out/tr_$v/b_kernel_trace.csv 15 > gpurun_out/tr_$v.txt 2>&1
  rm -f gpurun_out/tr_$v/b_kernel_trace.csv
  echo "== $v"; cat gpurun_out/tr_$v.txt
done
