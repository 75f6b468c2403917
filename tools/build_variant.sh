#!/bin/bash
# Build an A/B variant of libmlamg_hip.so with extra -D flags on spmv.hip (the other objects are
# the in-tree build's), for timing runs with MLAMG_LIB=<out>:
#   tools/build_variant.sh tools/variants/libmlamg_w6.so -DMLAMG_RP_WAVES=6
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$1
shift
mkdir -p "$(dirname "$OUT")"
TMP=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-gpu-rdc \
  -I"$ROOT/include" "$@" -x hip -c "$ROOT/ml-amg_amd/csrc/spmv.hip" -o "$TMP/spmv.hip.o"
OBJS=$(ls "$ROOT"/ml-amg_amd/build/*.o | grep -v '/spmv.hip.o$')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT" "$TMP/spmv.hip.o" $OBJS -lrccl
rm -rf "$TMP"
echo "built $OUT"
