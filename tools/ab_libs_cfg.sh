#!/bin/bash
# Interleaved A/B of prebuilt libldpc_nms variants over several SURVEY 8d configs (timing only):
#   CFGS="C3 C4" ROUNDS=2 bash tools/ab_libs_cfg.sh ab_libs/A.so ab_libs/B.so
set -o pipefail
cd "$(dirname "$0")/.."
L=ldpc_error_floor_amd/libldpc_nms.so
cp $L /tmp/lib_default.so
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in ${CFGS:-C2}; do
    for v in "$@"; do
      cp "$v" $L || exit 1
      timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline ${BENCH_EXTRA:-} > /tmp/ab_cfg.json || { cp /tmp/lib_default.so $L; exit 1; }
      python3 -c "import json;d=json.load(open('/tmp/ab_cfg.json'));print('$c', '$v', d['ms_per_step'], 'ms', d['value'], d['config']['kernel'])"
    done
  done
done
cp /tmp/lib_default.so $L
