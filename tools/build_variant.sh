#!/bin/bash
# Build an A/B variant of libmlamg_hip.so with extra -D flags on one source (default spmv.hip;
# SRC=batch.hip for another, SRC_PATH=<file> to compile a different copy of it); the other
# objects are the in-tree build's. Timing runs pick it with MLAMG_LIB=<out>:
#   tools/build_variant.sh tools/variants/libmlamg_w6.so -DMLAMG_RP_WAVES=6
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$1
shift
SRC=${SRC:-spmv.hip}
SRC_PATH=${SRC_PATH:-$ROOT/ml-amg_amd/csrc/$SRC}
mkdir -p "$(dirname "$OUT")"
TMP=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-gpu-rdc \
  -I"$ROOT/include" -I"$ROOT/ml-amg_amd/csrc" "$@" -x hip -c "$SRC_PATH" -o "$TMP/$SRC.o"
OBJS=$(ls "$ROOT"/ml-amg_amd/build/*.o | grep -v "/$SRC.o\$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT" "$TMP/$SRC.o" $OBJS -lrccl
rm -rf "$TMP"
echo "built $OUT"
