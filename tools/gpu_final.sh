# round-end check: full GPU suite, smoke, default bench, then the 320^2 two-level rocprofv3
# summary after the PCG rework. Each GPU step has its own time limit; a crash ends the script.
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_full.sh || exit 1
rm -rf gpurun_out/prof320b
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof320b -o p -- python tools/amg2v_large_phases.py 320 > gpurun_out/ph320b_prof.log 2>&1 || { echo prof-fail; tail -5 gpurun_out/ph320b_prof.log; exit 1; }
grep grid gpurun_out/ph320b_prof.log | cut -c1-20,300-700
