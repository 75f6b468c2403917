set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/amg2v_large_phases.py 320 > gpurun_out/ph320.log 2>&1 || { echo fail1; tail -20 gpurun_out/ph320.log; exit 1; }
cat gpurun_out/ph320.log | grep grid
rm -rf gpurun_out/prof320
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof320 -o p -- python tools/amg2v_large_phases.py 320 > gpurun_out/ph320_prof.log 2>&1 || { echo fail2; tail -5 gpurun_out/ph320_prof.log; exit 1; }
find gpurun_out/prof320 -name "*kernel_stats.csv"
