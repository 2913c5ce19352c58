#!/bin/bash
# Interleaved A/B/C... of libldpc_nms builds: bash tools/ab_multi.sh ROUNDS A.so B.so [C.so ...]
# (bench.py C2 defaults, 10 timed steps each; prints ms per step per build and round)
set -o pipefail
cd "$(dirname "$0")/.."
L=ldpc_error_floor_amd/libldpc_nms.so
R=$1; shift
cp $L /tmp/lib_default.so
for i in $(seq 1 $R); do
  for v in "$@"; do
    cp "$v" $L || exit 1
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > /tmp/bench_ab.json || { cp /tmp/lib_default.so $L; exit 1; }
    python -c "import json;d=json.load(open('/tmp/bench_ab.json'));print('$v', d['ms_per_step'])"
  done
done
cp /tmp/lib_default.so $L
