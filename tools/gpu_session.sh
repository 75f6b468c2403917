# ad-hoc GPU session (edited per experiment)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -v -m gpu --timeout 120 --timeout-method thread -k "singular or lsqr or amg_2_v" > gpurun_out/pt3.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/pt3.log | head -40
exit $rc
