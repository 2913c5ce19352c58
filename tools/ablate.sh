#!/bin/bash
# Diagnostic: time the fused kernel with phases removed (results invalid; timing only).
set -o pipefail
cd "$(dirname "$0")/.."
for ab in ${ABLATE_SET:-0 1 2 3 4 7}; do
  LDPC_DIAG_ABLATE=$ab timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --iters ${ITERS:-20} > gpurun_out/abl.json || exit 1
  AB=$ab python - <<'PY'
import json, os
d = json.load(open("gpurun_out/abl.json"))
print("ablate=" + os.environ["AB"], d["ms_per_step"], "ms", d["config"]["kernel"], d["fer_at_snr"]["fer_last"])
PY
done
