#!/bin/bash
# PMC counters of the bit-sliced kernel for several library variants / settings on one box:
#   bash tools/pmc_ab.sh "label|env settings|path/to/lib.so or -" ...
# Per variant: SQ instruction counts + GRBM (pass 1), LDS activity and bank conflicts (pass 2),
# wave / wait cycles (pass 3); summaries in gpurun_out/pmc_ab/<label>_<pass>.txt.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
L=ldpc_error_floor_amd/libldpc_nms.so
OUT=gpurun_out/pmc_ab
mkdir -p $OUT
cp $L $OUT/lib_default.so
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE"
G2="SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE GRBM_COUNT"
G3="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_BUSY_CU_CYCLES"
for v in "$@"; do
  IFS='|' read -r label envs lib <<< "$v"
  [ "$lib" != "-" ] && cp "$lib" $L
  e=(); [ -n "$envs" ] && read -ra e <<< "$envs"
  i=0
  for grp in "$G1" "$G2" "$G3"; do
    i=$((i+1))
    timeout -s KILL 120 env "${e[@]}" rocprofv3 --pmc $grp -d $OUT/${label}_$i -o run --output-format csv -- python3 tools/prof_decode.py --kernel auto --batch 1048576 --reps 3 --config C2 > $OUT/${label}_$i.log 2>&1 || { echo "pmc $label $i failed"; tail -5 $OUT/${label}_$i.log; cp $OUT/lib_default.so $L; exit 1; }
    python3 tools/pmc_summary.py $OUT/${label}_$i > $OUT/${label}_$i.txt 2>&1
  done
  [ "$lib" != "-" ] && cp $OUT/lib_default.so $L
  echo "== $label"; cat $OUT/${label}_*.txt | sed -n '/k_bs</,/^==/p' | grep -v "^==" | sort -u
done
