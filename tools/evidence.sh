#!/bin/bash
# Round evidence for the current build (one GPU call): per-config kernel-trace + PMC passes
# (tools/profile.sh) turned into profiles/<ROUND>/<TAG>/<CFG>/ and profiles/traffic_*.json (read
# by bench.py), then the default C2 bench line (with the CPU baseline) and a rocprofv3
# kernel-trace summary of that same bench command.
# usage: ROUND=r2 TAG=s1 CONFIGS="C2 C3 C4 C5" bash tools/evidence.sh   (scratch: gpurun_out/ev_<TAG>)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${TAG:-s}; B=1048576; ROUND=${ROUND:-r2}
OUT=gpurun_out/ev_$TAG
mkdir -p $OUT
for c in ${CONFIGS:-C2}; do
  K=auto B=$B TAG=$TAG CFG=$c bash tools/profile.sh || exit 1
  python3 tools/traffic_json.py gpurun_out/prof_${TAG}_${c}_auto --batch $B --out $OUT/$c > $OUT/traffic_$c.log || exit 1
  cp profiles/traffic_*.json $OUT/ 2>/dev/null
done
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 600 python3 bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail $OUT/bench_c2.err; exit 1; }
cat $OUT/bench_c2.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/bench_trace -o bench --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/bench_c2_traced.json 2> $OUT/bench_c2_traced.err || { tail $OUT/bench_c2_traced.err; exit 1; }
cat $OUT/bench_c2_traced.json
