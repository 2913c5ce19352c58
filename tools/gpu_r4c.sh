set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_traced.json 2> $O/bench_traced.err || exit 1
cat $O/bench_traced.json
for c in C3 C4 C5; do timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$c -o run --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit 1; python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c', d['value'], d['ms_per_step'], d['config']['kernel'], 'e2e', d['e2e_with_rng'])"; done
bash tools/gpu_session.sh r4c ab:C4:ab_libs/head.so,ab_libs/gbl1.so,default,env=LDPC_BS_LPC=4,env=LDPC_BS_INST=7:2 ab:C3:ab_libs/head.so,ab_libs/gbl1.so,default:2 ab:C2:ab_libs/head.so,default:3 || exit 1
K=flood CFG=C2 TAG=r4 B=1048576 bash tools/profile.sh || exit 1
K=auto CFG=C2 TAG=e2e PROF_EXTRA=--e2e bash tools/profile.sh || exit 1
