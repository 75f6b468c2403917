#!/bin/bash
# A build variant (tools/abv/libmlamg_$V.so): its parity tests (K = pytest -k expression), then the
# C4 bench alternating with the default library, then one traced cycle of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
MLAMG_LIB=$PWD/tools/abv/libmlamg_$V.so timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hierarchy.py tests/test_gpu_kernels.py -k "${K:-sorted or exact or c4_full or results_do_not}" > gpurun_out/r04/var_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/r04/var_tests.log; exit 1; }
tail -1 gpurun_out/r04/var_tests.log
exec_ab() { bash tools/gpu_r04_epf.sh; }
V=$V exec_ab
