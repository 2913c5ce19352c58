# round 4, session p: where C5's LDS bank conflicts come from — bsc diagnostic builds with one
# class of LDS accesses made conflict-free (results invalid; ldpc_bsc.hip BSC_DIAG bits, built
# from a patched copy: 1 check-phase Tv reads, 2 check-phase record reads, 4 check-phase
# sign/argmin words, 8 variable-phase sign/argmin words, 16 variable-phase record reads,
# 32 variable-phase Tv writes); LDS counters per build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4p; mkdir -p $O
L=ldpc_error_floor_amd/libldpc_nms.so
cp $L $O/.lib_default.so
for v in default bscd1 bscd2 bscd4 bscd8 bscd16 bscd32; do
  if [ $v = default ]; then cp $O/.lib_default.so $L; else cp ab_libs/$v.so $L; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $O/pmc_$v -o run --output-format csv -- python3 tools/prof_decode.py --kernel auto --batch 1048576 --reps 3 --config C5 > $O/pmc_$v.log 2>&1 || { cp $O/.lib_default.so $L; tail -5 $O/pmc_$v.log; exit 1; }
  echo "done $v"
done
cp $O/.lib_default.so $L
