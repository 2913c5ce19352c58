#!/bin/bash
# Build a libldpc_nms.so variant of the bit-sliced kernel (ldpc_bs.hip) for A/B runs, without
# touching the tree:   [BS_SRC=other/ldpc_bs.hip] bash tools/bs_variant.sh ab_libs/NAME.so [hipcc flags]
# (-DBS_DIAG compiles in the LDPC_DIAG_ABLATE phase switches, for timing ablations)
# Recompiles ldpc_bs.hip with the flags and links it with the in-tree objects of the other
# sources (build those first: python -m ldpc_error_floor_amd.build).  Compare with tools/ab_lib.sh.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=$1; shift
B=ldpc_error_floor_amd/_build
W=$(mktemp -d /tmp/ldpc_bsvar.XXXX)
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Ildpc_error_floor_amd/csrc -mllvm -pragma-unroll-threshold=500000 $*"
/opt/rocm/bin/hipcc $FLAGS -c ${BS_SRC:-ldpc_error_floor_amd/csrc/ldpc_bs.hip} -o "$W/bs.o"
objs=$(ls $B/*.o | grep -v "/ldpc_bs.o")
mkdir -p "$(dirname "$OUT")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $objs "$W/bs.o"
rm -rf "$W"
echo "$OUT"
