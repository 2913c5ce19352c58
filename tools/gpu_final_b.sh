# round-end evidence, part B: the companion config lines (C3-C5, all kernels) and the float
# modes on C2
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r5z}
OUT=gpurun_out/ev_$TAG; mkdir -p $OUT
CONFIGS="C3 C4 C5" bash tools/bench_configs.sh > $OUT/bench_configs.log 2>&1 || { tail -20 $OUT/bench_configs.log; exit 1; }
cp gpurun_out/bench_C3.json gpurun_out/bench_C4.json gpurun_out/bench_C5.json $OUT/
cut -c1-300 $OUT/bench_configs.log
for m in "--decoding-type 1" "--decoding-type 3" "--decoding-type 2 --q-bit 6"; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --all-kernels $m > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$m', d['value'], d['config']['kernel'], d['ms_per_step'], d.get('kernels'))"
  cat $OUT/b.json >> $OUT/bench_float_modes.jsonl
done
echo done
