#!/bin/bash
# Fence-free PCG: parity tests, then two-level amg_2_v with the PCG coarse solve (320^2, 512^2)
# against the previous build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu_coarse_pcg.py tests/test_gpu_preconditioner.py tests/test_gpu_batch.py > gpurun_out/r04/pcg_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/r04/pcg_tests.log; exit 1; }
tail -1 gpurun_out/r04/pcg_tests.log
timeout -k 10 300 python3 tools/amg2v_large.py 320 512 > gpurun_out/r04/pcg_new.log 2>&1 || { echo "new failed"; tail -5 gpurun_out/r04/pcg_new.log; exit 1; }
MLAMG_LIB=$PWD/tools/abv/libmlamg_pcgold.so timeout -k 10 300 python3 tools/amg2v_large.py 320 512 > gpurun_out/r04/pcg_old.log 2>&1 || { echo "old failed"; tail -5 gpurun_out/r04/pcg_old.log; exit 1; }
echo new; tail -3 gpurun_out/r04/pcg_new.log; echo old; tail -3 gpurun_out/r04/pcg_old.log
