#!/bin/bash
# Build a libldpc_nms.so variant of the fused v5 kernel for A/B runs, without touching the tree:
#   bash tools/build_variant.sh ab_libs/NAME.so [PATCH] [extra hipcc flags]
# Copies ldpc_error_floor_amd/csrc to a scratch dir, applies PATCH (a `git diff` of csrc files,
# applied with -p3 relative to csrc) if given, recompiles ldpc_fused5.hip and every per-shape unit
# in parallel and links them with the in-tree objects of the other sources (build those first:
# python -m ldpc_error_floor_amd.build).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=$1; shift
PATCH=${1:-}; [ $# -gt 0 ] && shift
B=ldpc_error_floor_amd/_build
W=$(mktemp -d /tmp/ldpc_variant.XXXX)
cp -r ldpc_error_floor_amd/csrc "$W/csrc"
# only the fused v5 units are rebuilt; a patch touching any other source (a shared header such as
# ldpc_internal.h changes struct layouts) would link mismatched objects: refuse it
if [ -n "$PATCH" ] && grep -E '^\+\+\+ ' "$PATCH" | grep -vqE 'ldpc_fused5(_kernel\.h|\.hip|_shape\.hip)$'; then
  echo "build_variant: $PATCH touches files other than ldpc_fused5*; build the full tree instead" >&2
  rm -rf "$W"; exit 2
fi
if [ -n "$PATCH" ]; then (cd "$W/csrc" && patch -s -p3 < "$OLDPWD/$PATCH"); fi
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude -I$W/csrc -mllvm -pragma-unroll-threshold=500000 $*"
NS=$(python3 -c "import sys; sys.path.insert(0, 'ldpc_error_floor_amd'); import build; print(build._f5_shape_count())")
/opt/rocm/bin/hipcc $FLAGS -c "$W/csrc/ldpc_fused5.hip" -o "$W/f5.o" &
for i in $(seq 0 $((NS - 1))); do
  /opt/rocm/bin/hipcc $FLAGS -DF5_SHAPE=$i -c "$W/csrc/ldpc_fused5_shape.hip" -o "$W/f5_s$i.o" &
done
wait
objs=$(ls $B/*.o | grep -v "ldpc_fused5")
mkdir -p "$(dirname "$OUT")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $objs "$W"/f5*.o
rm -rf "$W"
echo "$OUT"
