set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_traced.json 2> $O/bench_traced.err || exit 1
cat $O/bench_traced.json
for c in C3 C4 C5; do timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$c -o run --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit 1; python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c', d['value'], d['ms_per_step'], 'e2e', d['e2e_with_rng'])"; done
CONFIGS="" bash tools/gpu_session.sh r4c ab:C4:default,env=LDPC_BS_LPC=4,env=LDPC_BS_INST=6:2 || exit 1
K=flood CFG=C2 TAG=r4 B=1048576 bash tools/profile.sh || exit 1
K=auto CFG=C2 TAG=e2e PROF_EXTRA=--e2e bash tools/profile.sh || exit 1
bash tools/gpu_session.sh r4c ab:C2:default,ab_libs/gbl1.so:3 ab:C3:default,ab_libs/gbl1.so:2 ab:C4:default,ab_libs/gbl1.so:2 || exit 1
