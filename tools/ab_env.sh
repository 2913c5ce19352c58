#!/bin/bash
# Interleaved A/B of environment settings on the SURVEY 8d workloads (timing only):
#   CFGS="C4 C5" ROUNDS=2 bash tools/ab_env.sh "LDPC_F5_BALANCE=0" "LDPC_F5_BALANCE=1"
# ("-" = no extra setting).  Prints ms per step and the kernel for each (config, setting, round).
set -o pipefail
cd "$(dirname "$0")/.."
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in ${CFGS:-C2}; do
    for v in "$@"; do
      e=(); [ "$v" != "-" ] && read -ra e <<< "$v"
      env "${e[@]}" timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline > /tmp/ab_env.json || exit 1
      python3 -c "import json;d=json.load(open('/tmp/ab_env.json'));print('$c', '$v', d['ms_per_step'], 'ms', d['value'], d['config']['kernel'])"
    done
  done
done
