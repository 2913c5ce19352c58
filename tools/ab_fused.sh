#!/bin/bash
# GPU tests, then bench each fused-kernel variant in its own process.
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_ab.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_ab.log; [ $rc -ne 0 ] && exit $rc
run() { env $1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ab.json || exit 1; python -c "import json;d=json.load(open('gpurun_out/bench_ab.json'));print('$1', d['value'], d['config']['kernel'], d['ms_per_step'])"; }
for cfg in ${AB_CONFIGS:-"LDPC_FUSED_VERSION=3" "LDPC_FUSED_VERSION=4 LDPC_F4_SHAPE=0" "LDPC_FUSED_VERSION=4 LDPC_F4_SHAPE=1"}; do run "$cfg"; done
