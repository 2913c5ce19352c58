# round 4, session c: the channel fix on the GPU, the whole GPU suite, the traced benches
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 120 python -u profiles/r4/sessions/diag_r4.py > $O/diag.log 2>&1; rc=$?; cat $O/diag.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; grep -E "FAILED|^ERROR" $O/pytest_gpu.log | head -30
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_traced.json 2> $O/bench_traced.err || exit 1
cat $O/bench_traced.json
for c in C3 C4 C5; do timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$c -o run --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit 1; python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c', d['value'], d['ms_per_step'], d['config']['kernel'], 'e2e', d['e2e_with_rng'])"; done
