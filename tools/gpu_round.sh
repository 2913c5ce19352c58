#!/bin/bash
# One GPU-box session: parity tests, smoke, a short bench, and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r1}
BENCH_ARGS=${BENCH_ARGS:-"--steps 5 --warmup 2"}
echo "== pytest -m gpu" && timeout -k 10 600 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -5 $OUT/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && { echo "pytest failed rc=$rc"; exit $rc; }
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
echo "== bench" && timeout -k 10 600 python bench.py $BENCH_ARGS > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { cat $OUT/bench_$TAG.err | tail -20; exit 1; }
cat $OUT/bench_$TAG.json
if [ -n "$PROFILE" ]; then
  echo "== rocprofv3 kernel trace"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline $PROFILE_ARGS > $OUT/prof_$TAG.log 2>&1 || { tail -20 $OUT/prof_$TAG.log; exit 1; }
  find $OUT/prof_$TAG -name "*stats*" | head
fi
echo done
