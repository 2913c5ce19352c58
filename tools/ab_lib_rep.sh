#!/bin/bash
# Interleaved A/B of two libldpc_nms builds: bash tools/ab_lib_rep.sh A.so B.so [rounds]
set -o pipefail
cd "$(dirname "$0")/.."
L=ldpc_error_floor_amd/libldpc_nms.so
cp $L gpurun_out/lib_default.so
for i in $(seq 1 ${3:-3}); do
  for v in "$1" "$2"; do
    cp "$v" $L || exit 1
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ab.json || { cp gpurun_out/lib_default.so $L; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bench_ab.json'));print('$v', d['ms_per_step'])"
  done
done
cp gpurun_out/lib_default.so $L
