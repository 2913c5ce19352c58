#!/bin/bash
# One GPU-box check of the committed tree: GPU tests, smoke, the default bench line.
# Every GPU step has its own time limit; the chain stops at the first failure.
#   TAG=<name> bash tools/gpu_check.sh      (output under gpurun_out/<TAG>/)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-check}
mkdir -p $OUT
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
  ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
[ -n "$SKIP_BENCH" ] && exit 0
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
echo "== bench"
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
