#!/bin/bash
# Round-4 A/B session: fused amg_2_v (this tree vs the pre-Markstein batch.hip), the uniform
# row-pair kernel at 4 / 2 / 1 chunks per workgroup, and the C4 bench cycle with k_rowpair vs
# k_rowpat_uni (alternating). Each step bounded; the first failure ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
O=gpurun_out/ab
run() { local t=$1; shift; timeout -k 10 "$t" "$@" || { echo "step failed rc=$?: $*"; exit 1; }; }
run 200 python -u tools/amg2v_ab.py > $O/batch_new1.log 2>&1
MLAMG_LIB=$PWD/tools/abx/libbatch_old.so run 200 python -u tools/amg2v_ab.py > $O/batch_old.log 2>&1
run 200 python -u tools/amg2v_ab.py > $O/batch_new2.log 2>&1
for ch in 2 1; do MLAMG_RPU_CH=$ch run 200 python -u tools/rpuni_ab.py > $O/rpuni_ch$ch.log 2>&1; done
B="python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c3 --no-varcoef"
for rep in 1 2; do
  MLAMG_RP_UNI=0 run 300 $B > $O/bench_pair_$rep.log 2>&1
  MLAMG_RP_UNI=1 run 300 $B > $O/bench_uni4_$rep.log 2>&1
  MLAMG_RP_UNI=1 MLAMG_RPU_CH=2 run 300 $B > $O/bench_uni2_$rep.log 2>&1
done
for f in $O/batch_*.log; do echo "$f: $(grep '^{' $f)"; done
for f in $O/bench_*.log; do echo "$f: $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["avg_launch_us"], r["warm_avg_launch_us"], r["frac"], d["cycle_hbm_frac"])')"; done
