#!/bin/bash
# Round evidence for the default kernel: PMC profile + traffic JSON, the full bench line
# (with the CPU baseline), and a rocprofv3 kernel-trace summary of the bench command itself.
# usage: TAG=r1v5 bash tools/round_evidence.sh     (outputs under gpurun_out/)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${TAG:-r}; B=${B:-1048576}
K=fused B=$B TAG=$TAG bash tools/profile.sh || exit 1
python3 tools/traffic_json.py gpurun_out/prof_${TAG}_fused --batch $B --out gpurun_out/evidence_${TAG} || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/evidence_${TAG}/bench.json 2> gpurun_out/evidence_${TAG}/bench.err || { tail gpurun_out/evidence_${TAG}/bench.err; exit 1; }
cat gpurun_out/evidence_${TAG}/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/evidence_${TAG}/bench_trace -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/evidence_${TAG}/bench_traced.json 2> gpurun_out/evidence_${TAG}/bench_traced.err || { tail gpurun_out/evidence_${TAG}/bench_traced.err; exit 1; }
cat gpurun_out/evidence_${TAG}/bench_traced.json
