# round 4, session k: one-chunk UCN hard-decision addresses in LDS (C3 spill-free): whole suite,
# A/B on C3 against the previous build, C2 unchanged check
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; grep -E "FAILED|^ERROR" $O/pytest_gpu.log | head -30
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_session.sh r4k ab:C3:ab_libs/pre_hdl.so,ab_libs/btids0.so,default:2 ab:C2:ab_libs/pre_hdl.so,ab_libs/btids0.so,default:2 || exit 1
# (the pool is slow to give boxes: the round-end evidence of this same build follows in this call)
SKIP_TESTS=1 TAG=r4f bash tools/gpu_final_a.sh || exit 1
