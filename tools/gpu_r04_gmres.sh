#!/bin/bash
# GMRES with the device-side Arnoldi step: parity tests, then timing against the previous build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_preconditioner.py tests/test_gpu_coarse_pcg.py tests/test_gpu_callers.py > gpurun_out/r04/gm_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/r04/gm_tests.log; exit 1; }
tail -1 gpurun_out/r04/gm_tests.log
timeout -k 10 200 python3 tools/gmres_timing.py > gpurun_out/r04/gm_new.log 2>&1 || { echo "timing failed"; tail -5 gpurun_out/r04/gm_new.log; exit 1; }
MLAMG_LIB=$PWD/tools/abv/libmlamg_gmold.so timeout -k 10 200 python3 tools/gmres_timing.py > gpurun_out/r04/gm_old.log 2>&1 || { echo "timing old failed"; tail -5 gpurun_out/r04/gm_old.log; exit 1; }
echo new; grep gmres gpurun_out/r04/gm_new.log; echo old; grep gmres gpurun_out/r04/gm_old.log
