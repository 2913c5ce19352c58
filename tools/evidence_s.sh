#!/bin/bash
# Round evidence for the current build (one GPU call): per-config PMC + kernel-trace passes
# (tools/profile.sh), the traffic/VALU JSON bench.py reads, the full C2 bench line (with the CPU
# baseline), and a rocprofv3 kernel-trace summary of the bench command itself.
# usage: TAG=s4 bash tools/evidence_s.sh        (outputs under gpurun_out/ev_<TAG>/)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${TAG:-s}; B=1048576
OUT=gpurun_out/ev_$TAG
mkdir -p $OUT
for c in ${CONFIGS:-C2 C4 C5 C3}; do
  K=fused B=$B TAG=${TAG}${c} CFG=$c bash tools/profile.sh || exit 1
  python3 tools/traffic_json.py gpurun_out/prof_${TAG}${c}_fused --batch $B --out $OUT/$c > $OUT/traffic_$c.log || exit 1
done
timeout -k 10 600 python3 bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail $OUT/bench_c2.err; exit 1; }
cat $OUT/bench_c2.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/bench_trace -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c2_traced.json 2> $OUT/bench_c2_traced.err || { tail $OUT/bench_c2_traced.err; exit 1; }
cat $OUT/bench_c2_traced.json
