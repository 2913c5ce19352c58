#!/bin/bash
# Build a libldpc_nms.so variant of the bit-sliced kernel instances (ldpc_bs_inst.hip, one unit
# per kBsInst entry) for A/B runs, without touching the tree:
#   bash tools/bs_variant.sh ab_libs/NAME.so [hipcc flags]
# (-DBS_DIAG compiles in the LDPC_DIAG_ABLATE phase switches, for timing ablations)
# Recompiles the instance units (and the bsc and bsl host units) with the flags and links them with the in-tree objects of the
# other sources (build those first: python -m ldpc_error_floor_amd.build).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=$1; shift
B=ldpc_error_floor_amd/_build
W=$(mktemp -d /tmp/ldpc_bsvar.XXXX)
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Ildpc_error_floor_amd/csrc -mllvm -pragma-unroll-threshold=500000 $*"
N=$(ls $B/ldpc_bs_i*.o | wc -l)
for i in $(seq 0 $((N - 1))); do
  /opt/rocm/bin/hipcc $FLAGS -mllvm -amdgpu-use-amdgpu-trackers -DBS_INST=$i -c ldpc_error_floor_amd/csrc/ldpc_bs_inst.hip -o "$W/bs_i$i.o" &
done
/opt/rocm/bin/hipcc $FLAGS -c ldpc_error_floor_amd/csrc/ldpc_bsc.hip -o "$W/bsc.o" &
/opt/rocm/bin/hipcc $FLAGS -c ldpc_error_floor_amd/csrc/ldpc_bs.hip -o "$W/bsh.o" &
wait
objs=$(ls $B/*.o | grep -v "/ldpc_bs_i[0-9]*\.o" | grep -v "/ldpc_bsc\.o" | grep -v "/ldpc_bs\.o")
mkdir -p "$(dirname "$OUT")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $objs $W/bs_i*.o $W/bsc.o $W/bsh.o
rm -rf "$W"
echo "$OUT"
