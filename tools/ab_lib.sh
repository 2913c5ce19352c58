#!/bin/bash
# A/B of prebuilt libldpc_nms variants: usage  bash tools/ab_lib.sh VARIANT.so [VARIANT2.so ...]
# (each file is copied over ldpc_error_floor_amd/libldpc_nms.so in turn; the default build is
#  benched first and restored at the end)
set -o pipefail
cd "$(dirname "$0")/.."
L=ldpc_error_floor_amd/libldpc_nms.so
cp $L gpurun_out/lib_default.so
bench() { timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ab.json || return 1; python -c "import json;d=json.load(open('gpurun_out/bench_ab.json'));print('$1', d['value'], d['config']['kernel'], d['ms_per_step'])"; }
bench default || exit 1
for v in "$@"; do cp "$v" $L && bench "$v" || { cp gpurun_out/lib_default.so $L; exit 1; }; done
cp gpurun_out/lib_default.so $L
