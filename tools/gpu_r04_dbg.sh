#!/bin/bash
# Streaming calibration + timing-only k_rowpat_uni variants (what each part of the kernel costs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/stream_calib.py > gpurun_out/r04/stream_calib.log 2>&1 || { echo "calib failed rc=$?"; tail -5 gpurun_out/r04/stream_calib.log; exit 1; }
cat gpurun_out/r04/stream_calib.log
for v in 1 2 4 8 15; do
  MLAMG_LIB=$PWD/tools/abv/libmlamg_dbg$v.so timeout -k 10 200 python3 tools/rpuni_sweep.py 216 ch=4,pad=0 ch=2,pad=0 > gpurun_out/r04/dbg$v.log 2>&1 || { echo "dbg$v failed rc=$?"; tail -5 gpurun_out/r04/dbg$v.log; exit 1; }
  echo "dbg$v"; grep ch= gpurun_out/r04/dbg$v.log
done
