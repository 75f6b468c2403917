# ad-hoc GPU session (edited per experiment)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pt_batch.log 2>&1 || { tail -30 gpurun_out/pt_batch.log; exit 1; }
tail -3 gpurun_out/pt_batch.log
MLAMG_BATCH_TIMING=1 timeout -k 10 400 python -u tools/amg2v_timing.py --out gpurun_out/amg2v_timing.json > gpurun_out/amg2v_timing.log 2>&1 || { tail -30 gpurun_out/amg2v_timing.log; exit 1; }
grep -v "problem [0-9]" gpurun_out/amg2v_timing.log | tail -20
grep "problem 4[5-7]" gpurun_out/amg2v_timing.log
