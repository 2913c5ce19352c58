#!/usr/bin/env python3
"""Register use, spills and static instruction counts of every kernel in one translation unit
(device-only assembly), for before/after checks of a kernel edit without a GPU:

    python3 tools/kstats.py ldpc_bs_inst.hip -DBS_INST=0 [-DBS_KEEP=4 ...]
    python3 tools/kstats.py ldpc_bsc.hip

Prints per kernel: VGPRs, SGPRs, VGPR/SGPR spills, LDS (static), and the number of VALU / LDS /
global / scalar-memory instructions in the ISA (static counts, not per-iteration costs)."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ldpc_error_floor_amd", "csrc")


def main():
    src = sys.argv[1]
    if not os.path.exists(src):
        src = os.path.join(CSRC, src)
    defs = sys.argv[2:]
    out = os.path.join(tempfile.mkdtemp(prefix="kstats"), "k.s")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
           "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "-mllvm", "-pragma-unroll-threshold=500000",
           "--cuda-device-only", "-S", "-o", out, src] + defs
    subprocess.run(cmd, check=True)
    s = open(out).read()
    # instruction counts per function body
    bodies = {}
    cur = None
    for line in s.splitlines():
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            cur = m.group(1)
            bodies[cur] = []
            continue
        if cur and line.startswith("\t") and not line.strip().startswith((";", ".")):
            bodies[cur].append(line.strip().split()[0])
        if line.startswith(".Lfunc_end"):
            cur = None
    for e in s.split("\n  - ."):
        n = re.search(r"\.name:\s+(\S+)", e)
        if not n or not n.group(1).startswith("_Z"):
            continue
        name = n.group(1)
        g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", e) or [None, "?"])[1]   # noqa: E731
        ops = bodies.get(name, [])
        valu = sum(1 for o in ops if o.startswith("v_"))
        lds = sum(1 for o in ops if o.startswith("ds_"))
        glb = sum(1 for o in ops if o.startswith(("global_", "buffer_", "flat_", "scratch_")))
        smem = sum(1 for o in ops if o.startswith("s_load") or o.startswith("s_buffer_load"))
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        print(f"{dem[:110]}\n   vgpr {g('vgpr_count')} agpr {g('agpr_count')} sgpr {g('sgpr_count')} "
              f"vspill {g('vgpr_spill_count')} sspill {g('sgpr_spill_count')} lds {g('group_segment_fixed_size')} "
              f"| VALU {valu} LDS {lds} VMEM {glb} SMEM {smem} total {len(ops)}")


if __name__ == "__main__":
    main()
