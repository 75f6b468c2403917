#!/bin/bash
# k_rowpat_uni launch-shape / store-hint sweep (cold dispatch-packet timing) and a quick bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
C="ch=4,pad=0 ch=4,pad=6000 ch=4,pad=12000 ch=4,pad=20200 ch=4,pad=33800 ch=4,pad=61200 ch=2,pad=0 ch=1,pad=0 ch=2,pad=20000"
timeout -k 10 300 python3 tools/rpuni_sweep.py 216 $C > gpurun_out/r04/sweep_default.log 2>&1 || { echo "sweep failed rc=$?"; tail -5 gpurun_out/r04/sweep_default.log; exit 1; }
cat gpurun_out/r04/sweep_default.log
MLAMG_LIB=$PWD/tools/abv/libmlamg_nt.so timeout -k 10 300 python3 tools/rpuni_sweep.py 216 ch=4,pad=0 ch=4,pad=12000 ch=4,pad=20200 ch=2,pad=0 > gpurun_out/r04/sweep_nt.log 2>&1 || { echo "sweep nt failed rc=$?"; tail -5 gpurun_out/r04/sweep_nt.log; exit 1; }
cat gpurun_out/r04/sweep_nt.log
timeout -k 10 300 python3 bench.py --steps 50 --no-cpu-baseline --no-c3 --no-varcoef > gpurun_out/r04/bench_timer.log 2>&1 || { echo "bench failed rc=$?"; tail -5 gpurun_out/r04/bench_timer.log; exit 1; }
grep '^{' gpurun_out/r04/bench_timer.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["avg_launch_us"], r["median_launch_us"], r["stream_event_avg_launch_us"], r["warm_avg_launch_us"], r["frac"])'
