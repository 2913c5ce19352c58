#!/bin/bash
# rocprofv3 passes for one kernel: kernel trace + stats, then PMC counters (one group per
# pass, at most 8 SQ / 4 TCC / 2 GRBM counters each; counters never combined with tracing
# domains).  Output under gpurun_out/prof_<TAG>_<K>; tools/traffic_json.py turns it into
# profiles/<round>/... and profiles/traffic_<kernel>.json.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
K=${K:-auto}; B=${B:-1048576}; TAG=${TAG:-p}; CFG=${CFG:-C2}
OUT=gpurun_out/prof_${TAG}_${CFG}_${K}
mkdir -p $OUT
ARGS="--kernel $K --batch $B --reps 3 --config $CFG ${PROF_EXTRA:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/prof_decode.py $ARGS > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_BUSY_CU_CYCLES" \
           "SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 tools/prof_decode.py $ARGS > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
echo profiled $CFG $K
