#!/bin/bash
# rocprofv3 passes for one kernel: kernel trace + stats, then PMC counters (one group per
# pass; counters never combined with tracing domains).  Output under gpurun_out/prof_<TAG>.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
K=${K:-fused}; B=${B:-262144}; TAG=${TAG:-p}
OUT=gpurun_out/prof_${TAG}_${K}
mkdir -p $OUT
ARGS="--kernel $K --batch $B --reps 3 --config ${CFG:-C2}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/prof_decode.py $ARGS > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 tools/prof_decode.py $ARGS > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
echo profiled $K
