# PCG coarse solve: GPU tests of the coarse solver, then the 320^2 / 512^2 two-level setup /
# cycle split (defaults). Each GPU step has its own time limit; a failure ends the script.
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_coarse_pcg.py > gpurun_out/pcg_tests.log 2>&1 || { echo tests-fail; tail -30 gpurun_out/pcg_tests.log; exit 1; }
tail -1 gpurun_out/pcg_tests.log
MLAMG_TIMING=1 timeout -k 10 300 python -u tools/amg2v_large_phases.py 320 512 > gpurun_out/pcg_phases.log 2>&1 || { echo ph-fail; tail -20 gpurun_out/pcg_phases.log; exit 1; }
grep grid gpurun_out/pcg_phases.log | cut -c1-20,250-900
grep "gs_create" gpurun_out/pcg_phases.log | tail -24
