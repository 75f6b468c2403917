# ad-hoc GPU session (edited per experiment)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gnn.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pt_gnn.log 2>&1 || { tail -40 gpurun_out/pt_gnn.log; exit 1; }
tail -3 gpurun_out/pt_gnn.log
