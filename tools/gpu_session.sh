# ad-hoc GPU session (edited per experiment)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "dense or two_level or amg_2_v" > gpurun_out/pt_dense.log 2>&1 || { tail -40 gpurun_out/pt_dense.log; exit 1; }
tail -3 gpurun_out/pt_dense.log
timeout -k 10 300 python tools/amg2v_phases.py 2>&1 | grep -v amdgpu
