#!/bin/bash
# Interleaved A/B of the decode-only and the sweep-step (e2e, channel generated per step) rates:
#   bash tools/e2e_ab.sh ab_libs/VARIANT.so [configs] [rounds]
# prints "config lib decode-ms e2e-ms e2e/decode" per run (GPU box; restores the default lib)
set -o pipefail
cd "$(dirname "$0")/.."
V=$1; CFGS=${2:-C2 C3}; R=${3:-2}
L=ldpc_error_floor_amd/libldpc_nms.so
mkdir -p gpurun_out
cp $L gpurun_out/.lib_default.so
for r in $(seq 1 $R); do
  for v in default $V; do
    if [ $v = default ]; then cp gpurun_out/.lib_default.so $L; else cp $v $L; fi
    for c in $CFGS; do
      timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/e2e.json 2> gpurun_out/e2e.err || { tail -5 gpurun_out/e2e.err; cp gpurun_out/.lib_default.so $L; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/e2e.json'));print('$c $v', d['ms_per_step'], d['e2e_with_rng']['ms_per_step'], round(d['e2e_with_rng']['codewords_per_s']/d['value'],4))"
    done
  done
done
cp gpurun_out/.lib_default.so $L
