# round 4, session e: the inline-threshold channel sampler on the GPU (whole suite), C2 bench
# with the end-to-end rate, the flood bench line, LLR-load A/B on the one-workgroup-per-CU C4
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 120 python -u profiles/r4/sessions/diag_r4.py > $O/diag.log 2>&1; rc=$?; cat $O/diag.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; grep -E "FAILED|^ERROR" $O/pytest_gpu.log | head -30
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_C2.json 2> $O/bench_C2.err || exit 1
cat $O/bench_C2.json
timeout -k 10 300 python3 bench.py --kernel flood --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_flood.json 2> $O/bench_flood.err || exit 1
cat $O/bench_flood.json
bash tools/gpu_session.sh r4e ab:C4:ab_libs/llrall.so,ab_libs/afix.so,default,env=LDPC_BS_STAGGER=50,env=LDPC_BS_STAGGER=200:2 ab:C2:ab_libs/afix.so,default:2 || exit 1
