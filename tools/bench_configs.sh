#!/bin/bash
# The SURVEY §8 d workloads C2..C5 on one GPU (C2 = the driver's line); one JSON line each.
set -o pipefail
cd "$(dirname "$0")/.."
for c in ${CONFIGS:-C2 C3 C4 C5}; do
  timeout -k 10 600 python bench.py --config $c --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --all-kernels > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -5 gpurun_out/bench_$c.err; exit 1; }
  python - "$c" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/bench_{sys.argv[1]}.json"))
print(sys.argv[1], d["metric"], "|", d["value"], "cw/s", d["ms_per_step"], "ms", d["config"]["kernel"],
      "| e2e", d["e2e_with_rng"]["codewords_per_s"], "| others", d.get("kernels"), "| FER", d["fer_at_snr"]["fer_last"])
PY
done
