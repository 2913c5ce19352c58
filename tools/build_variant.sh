#!/bin/bash
# Build a libldpc_nms.so variant whose fused5 kernel comes from another source file (A/B runs):
#   bash tools/build_variant.sh path/to/ldpc_fused5_variant.hip ab_libs/NAME.so [extra hipcc flags]
# The other objects are the current in-tree build (python -m ldpc_error_floor_amd.build first).
set -euo pipefail
cd "$(dirname "$0")/.."
SRC=$1; OUT=$2; shift 2
B=ldpc_error_floor_amd/_build
mkdir -p "$(dirname "$OUT")" /tmp/ldpc_variant
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude \
  -Ildpc_error_floor_amd/csrc "$@" -c "$SRC" -o /tmp/ldpc_variant/f5.o
objs=$(ls $B/*.o | grep -v ldpc_fused5.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $objs /tmp/ldpc_variant/f5.o
echo "$OUT"
