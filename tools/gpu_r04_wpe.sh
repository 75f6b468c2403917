#!/bin/bash
# k_rowpat_uni at a forced 7 / 8 waves per SIMD (MLAMG_UNI_WPE builds): cold/warm sweep, then
# the C4 bench with each (alternating, same box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
for v in default wpe7 wpe8; do
  if [ $v = default ]; then unset MLAMG_LIB; else export MLAMG_LIB=$PWD/tools/abv/libmlamg_$v.so; fi
  timeout -k 10 200 python3 tools/rpuni_sweep.py 216 rpm=0,ch=4 rpm=0,ch=2 > gpurun_out/r04/wpe_$v.log 2>&1 || { echo "$v failed rc=$?"; tail -5 gpurun_out/r04/wpe_$v.log; exit 1; }
  echo $v; grep ch= gpurun_out/r04/wpe_$v.log
done
unset MLAMG_LIB
val() { grep '^{' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
B="python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-c3 --no-varcoef"
for i in 1 2; do
  timeout -k 10 300 $B > gpurun_out/r04/wb_a.log 2>&1 || exit 1; echo "default ch4 $(val gpurun_out/r04/wb_a.log)"
  MLAMG_RPU_CH=2 timeout -k 10 300 $B > gpurun_out/r04/wb_b.log 2>&1 || exit 1; echo "default ch2 $(val gpurun_out/r04/wb_b.log)"
  MLAMG_LIB=$PWD/tools/abv/libmlamg_wpe8.so MLAMG_RPU_CH=2 timeout -k 10 300 $B > gpurun_out/r04/wb_c.log 2>&1 || exit 1; echo "wpe8 ch2 $(val gpurun_out/r04/wb_c.log)"
  MLAMG_LIB=$PWD/tools/abv/libmlamg_wpe7.so timeout -k 10 300 $B > gpurun_out/r04/wb_d.log 2>&1 || exit 1; echo "wpe7 ch4 $(val gpurun_out/r04/wb_d.log)"
  MLAMG_LIB=$PWD/tools/abv/libmlamg_nt.so timeout -k 10 300 $B > gpurun_out/r04/wb_e.log 2>&1 || exit 1; echo "nt ch4 $(val gpurun_out/r04/wb_e.log)"
done
