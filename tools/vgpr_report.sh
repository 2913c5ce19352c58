#!/bin/bash
# VGPR count and spills of every fused v5 kernel build of one shape:  bash tools/vgpr_report.sh SHAPE
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p /tmp/ldpc_isa
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -Ildpc_error_floor_amd/csrc \
  -mllvm -pragma-unroll-threshold=500000 -DF5_SHAPE=$1 --cuda-device-only -S \
  -o /tmp/ldpc_isa/s$1.s ldpc_error_floor_amd/csrc/ldpc_fused5_shape.hip
python3 - /tmp/ldpc_isa/s$1.s <<'PY'
import re, subprocess, sys
s = open(sys.argv[1]).read()
for e in s.split("\n  - ."):
    n = re.search(r"\.name:\s+(\S+)", e)
    if not n or "k_fused5" not in n.group(1):
        continue
    v = re.search(r"\.vgpr_count:\s+(\d+)", e).group(1)
    sp = re.search(r"\.vgpr_spill_count:\s+(\d+)", e).group(1)
    name = subprocess.run(["c++filt", n.group(1)], capture_output=True, text=True).stdout
    print(name.split("k_fused5")[1].split("(")[0], "vgpr", v, "spill", sp)
PY
