#!/bin/bash
# Round-end evidence in one GPU call: pytest -m gpu + smoke (gpu_session), kernel-trace + PMC of
# C2-C5 with the default bench line and its rocprofv3 summary (evidence.sh), then the C3-C5 and
# float-mode lines (gpu_final_b.sh).  Output: gpurun_out/ev_$TAG (+ gpurun_out/$TAG for the tests).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-r5f}
bash tools/gpu_session.sh $TAG tests smoke || exit 1
TAG=$TAG ROUND=r5 CONFIGS="C2 C3 C4 C5" bash tools/evidence.sh > gpurun_out/ev_$TAG.log 2>&1 || { tail -20 gpurun_out/ev_$TAG.log; exit 1; }
tail -2 gpurun_out/ev_$TAG.log | cut -c1-300
TAG=$TAG bash tools/gpu_final_b.sh > gpurun_out/ev_${TAG}_b.log 2>&1 || { tail -20 gpurun_out/ev_${TAG}_b.log; exit 1; }
tail -7 gpurun_out/ev_${TAG}_b.log | cut -c1-300
