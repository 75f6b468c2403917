#!/bin/bash
# Plane-marching stencil kernel: parity tests, then the cold/warm sweep against k_rowpat_uni.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hierarchy.py -k "rowpat" > gpurun_out/r04/march_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/r04/march_tests.log; exit 1; }
tail -3 gpurun_out/r04/march_tests.log
timeout -k 10 300 python3 tools/rpuni_sweep.py 216 ${SWEEP:-rpm=0 rpm=1,mch=4 rpm=1,mch=2 rpm=1,mch=4,seg=5 rpm=1,mch=4,seg=20 rpm=1,mch=2,seg=5 rpm=1,mch=2,seg=20 rpm=1,mch=1 rpm=1,mch=1,seg=5 rpm=1,mch=1,seg=20 rpm=1,mch=2,pf=2 rpm=1,mch=1,pf=2 rpm=1,mch=2,pf=2,seg=20 rpm=1,mch=1,pf=2,seg=20} > gpurun_out/r04/march_sweep.log 2>&1 || { echo "sweep failed rc=$?"; tail -5 gpurun_out/r04/march_sweep.log; exit 1; }
cat gpurun_out/r04/march_sweep.log
