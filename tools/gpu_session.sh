#!/bin/bash
# One GPU-box session made of named steps; every GPU step has its own time limit and the session
# stops at the first failure (a fault, a timeout or a failing test ends it: nothing is retried).
#   bash tools/gpu_session.sh TAG STEP [STEP ...]        (output: gpurun_out/TAG/)
# steps:
#   tests                      pytest -m gpu (-rs: skips named) -> pytest_gpu.log
#   smoke                      __graft_entry__.smoke()
#   bench                      default bench.py line (C2, with the CPU baseline) -> bench_c2.json
#   configs                    bench.py --config C3 / C4 / C5 -> bench_C*.json
#   ab:CFG:A.so,B.so:ROUNDS    interleaved A/B of libldpc_nms builds on one config (ms per step)
#   ablate:CFG:LIB:SET         -DBS_DIAG build, LDPC_DIAG_ABLATE over SET (comma list), timing only
#   trace                      rocprofv3 kernel-trace summary of the default bench command
#   prof:CFG                   tools/profile.sh kernel trace + PMC passes of one config
#   tscale:CFG:T1,T2,...       ms per decode at each iteration count
#   uncor:CFG                  sweep rate with and without the uncorrected-word collection
#   stamp:CFG:LIB[:NAME=VALUE] per-wave phase clocks of a -DBS_STAMP build (optionally with an env switch)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
L=ldpc_error_floor_amd/libldpc_nms.so
cp $L $OUT/.lib_default.so
restore() { cp $OUT/.lib_default.so $L; }
bench_ms() {   # config, extra args -> prints "ms kernel value"
  timeout -k 10 300 python bench.py --config $1 --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-companions $2 > $OUT/.ab.json 2> $OUT/.ab.err || { tail -5 $OUT/.ab.err; return 1; }
  python -c "import json;d=json.load(open('$OUT/.ab.json'));print(d['ms_per_step'], d['config']['kernel'], d['value'], d['counters']['frame_err_last'], 'e2e', d['e2e_with_rng']['ms_per_step'])"
}
for step in "$@"; do
  echo "== $step $(date +%T)"
  IFS=: read -r kind a1 a2 a3 <<< "$step"
  case $kind in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
      rc=$?; tail -n 15 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && { echo "tests rc=$rc"; exit $rc; } ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
      cat $OUT/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail $OUT/bench_c2.err; exit 1; }
      cat $OUT/bench_c2.json ;;
    configs)
      for c in ${CONFIGS:-C3 C4 C5}; do
        timeout -k 10 600 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail $OUT/bench_$c.err; exit 1; }
        python -c "import json;d=json.load(open('$OUT/bench_$c.json'));print('$c', d['value'], d['ms_per_step'], d['config']['kernel'], 'e2e', d['e2e_with_rng']['codewords_per_s'])"
      done ;;
    ab)
      # variants: default | path/to/lib.so | env=NAME=VALUE (the default build with NAME set) |
      # default@NAME=VALUE | path/to/lib.so@NAME=VALUE
      for r in $(seq 1 ${a3:-2}); do
        for v in ${a2//,/ }; do
          envset=""
          if [ "${v#*@}" != "$v" ]; then envset=${v#*@}; v=${v%%@*}; fi   # LIB@NAME=VALUE
          if [ "$v" = default ]; then restore
          elif [ "${v#env=}" != "$v" ]; then restore; envset=${v#env=}
          else cp $v $L || exit 1; fi
          echo -n "$a1 $v${envset:+@$envset}: "
          if [ -n "$envset" ]; then ( export "$envset"; bench_ms $a1 ) || { restore; exit 1; }
          else bench_ms $a1 || { restore; exit 1; }; fi
        done
      done
      restore ;;
    ablate)
      cp $a2 $L || exit 1
      for ab in ${a3//,/ }; do
        echo -n "$a1 ablate=$ab: "; LDPC_DIAG_ABLATE=$ab bench_ms $a1 || { restore; exit 1; }
      done
      restore ;;
    uncor)
      # uncor:CFG  the collection sweep's rate against the plain sweep (tools/sweep_c5.py --uncor)
      # (the Uncor files stay on the box's /tmp: only the sweep JSON comes back)
      for u in "" "--uncor"; do
        d=/tmp/r6uncor_$a1${u:+_u}; rm -rf $d
        timeout -k 10 600 python tools/sweep_c5.py --config $a1 --deep-snrs ${UNCOR_SNRS:-3.0,3.5} --deep ${UNCOR_N:-4194304} --batch 1048576 $u --out $d > $OUT/uncor_$a1${u:+_u}.log 2>&1 || { tail -5 $OUT/uncor_$a1${u:+_u}.log; exit 1; }
        cp $d/sweep_*.json $OUT/uncor_$a1${u:+_u}.json; ls -la $d >> $OUT/uncor_$a1${u:+_u}.log
        tail -1 $OUT/uncor_$a1${u:+_u}.log
      done ;;
    tscale)
      # tscale:CFG:T1,T2,...  ms per decode at each iteration count (slope = per iteration,
      # intercept = the per-pack prologue / epilogue's throughput cost)
      for T in ${a2//,/ }; do echo -n "$a1 T=$T: "; bench_ms $a1 "--iters $T" || exit 1; done ;;
    stamp)
      # stamp:CFG:LIB[:NAME=VALUE]  a -DBS_STAMP build's per-wave phase clocks (stderr) -> stamp_CFG*.log
      cp $a2 $L || exit 1
      log=$OUT/stamp_${a1}${a3:+_${a3//[=]/_}}.log
      ( [ -n "$a3" ] && export "$a3"; timeout -k 10 300 python bench.py --config $a1 --steps 3 --warmup 1 --no-cpu-baseline > $log.json 2> $log ) || { restore; tail -5 $log; exit 1; }
      restore; grep -A17 "bs_stamp" $log | tail -18 ;;
    trace)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/bench_trace -o bench --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/bench_c2_traced.json 2> $OUT/bench_c2_traced.err || { tail $OUT/bench_c2_traced.err; exit 1; }
      cat $OUT/bench_c2_traced.json ;;
    prof)
      K=auto B=1048576 TAG=$TAG CFG=$a1 bash tools/profile.sh || exit 1
      python3 tools/traffic_json.py gpurun_out/prof_${TAG}_${a1}_auto --batch 1048576 --out $OUT/$a1 > $OUT/traffic_$a1.log || exit 1
      cp profiles/traffic_*.json $OUT/ 2>/dev/null; tail -n 20 $OUT/traffic_$a1.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session $TAG done $(date +%T)"
