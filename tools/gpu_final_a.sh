# round-end evidence, part A (the committed build; replaces round_evidence.sh): pytest -m gpu, smoke, per-config kernel
# trace + PMC passes (tools/evidence.sh -> traffic JSON for bench.py), the default bench line
# with the CPU baseline and its rocprofv3 kernel-trace summary -> gpurun_out/ev_$TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r5z}
OUT=gpurun_out/ev_$TAG; mkdir -p $OUT
rc=0
[ -n "$SKIP_TESTS" ] || { timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; grep -E "FAILED|^ERROR" $OUT/pytest_gpu.log | head -20; }
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
TAG=$TAG ROUND=r5 CONFIGS="C2 C3 C4 C5" bash tools/evidence.sh > $OUT/evidence.log 2>&1 || { tail -20 $OUT/evidence.log; exit 1; }
grep -h '"kernel"' $OUT/traffic_C*.log | cut -c1-200
cut -c1-400 $OUT/bench_c2.json
