#!/bin/bash
# Phase diagnostics of the fused kernel on one SURVEY 8d workload: per-workgroup stamps and
# phase ablations (timing only).  usage: CFG=C4 bash tools/diag_config.sh   (-> gpurun_out/)
set -o pipefail
cd "$(dirname "$0")/.."
CFG=${CFG:-C2}; B=${B:-1048576}
mkdir -p gpurun_out
LDPC_DIAG_STAMPS=gpurun_out/st_$CFG.bin timeout -k 10 200 python bench.py --config $CFG --batch $B --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/st_$CFG.json || exit 1
NB=$(python3 -c "import json;d=json.load(open('gpurun_out/st_$CFG.json'));k=d['config']['kernel'];import re;cw=int(re.search(r'cw(\d+)',k).group(1));print(($B+cw-1)//cw)")
T=$(python3 -c "import json;print(json.load(open('gpurun_out/st_$CFG.json'))['config']['iterations'])")
python3 tools/stamps.py gpurun_out/st_$CFG.bin --nblocks $NB --T $T > gpurun_out/stamps_$CFG.txt || exit 1
rm -f gpurun_out/st_$CFG.bin
for ab in ${ABLATE_SET:-0 1 2 4 7}; do
  LDPC_DIAG_ABLATE=$ab timeout -k 10 300 python bench.py --config $CFG --batch $B --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/abl.json || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/abl.json'));print('$CFG ablate=$ab', d['ms_per_step'], 'ms', d['config']['kernel'])"
done
