#!/bin/bash
# End-of-round evidence for the committed build in one GPU call (each step time-limited, the
# chain stops at the first failure):
#   1. pytest -m gpu (log), smoke()
#   2. per-config rocprofv3 kernel trace + PMC passes (tools/evidence.sh: C2..C5) -> traffic JSON,
#      then the default C2 bench line (CPU baseline included) and the rocprofv3 trace of it
#   3. the companion config lines (tools/bench_configs.sh, with the other kernels beside them)
#   4. the float-mode lines (ffl) on C2
# Everything lands in gpurun_out/ev_<TAG>/; copy it to profiles/<ROUND>/<TAG>/ afterwards.
#   TAG=f bash tools/round_evidence.sh
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${TAG:-f}
OUT=gpurun_out/ev_$TAG
mkdir -p $OUT
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
echo "== PMC + bench (C2..C5)"
TAG=$TAG CONFIGS="${CONFIGS:-C2 C3 C4 C5}" bash tools/evidence.sh > $OUT/evidence.log 2>&1 || { tail -20 $OUT/evidence.log; exit 1; }
grep -h '"kernel"' $OUT/traffic_C*.log | cut -c1-200
echo "== config lines"
CONFIGS="C3 C4 C5" bash tools/bench_configs.sh > $OUT/bench_configs.log 2>&1 || { tail -20 $OUT/bench_configs.log; exit 1; }
cp gpurun_out/bench_C3.json gpurun_out/bench_C4.json gpurun_out/bench_C5.json $OUT/
cut -c1-300 $OUT/bench_configs.log
echo "== float modes (ffl)"
for m in "--decoding-type 1" "--decoding-type 3" "--decoding-type 2 --q-bit 6"; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --all-kernels $m > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$m', d['value'], d['config']['kernel'], d['ms_per_step'], d.get('kernels'))"
  cat $OUT/b.json >> $OUT/bench_float_modes.jsonl
done
echo done
