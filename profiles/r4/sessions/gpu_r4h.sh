# round 4, session h: the opaque lane variable (BS_VVO) on the multi-chunk instances: whole
# suite, A/B on C4
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; grep -E "FAILED|^ERROR" $O/pytest_gpu.log | head -30
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_session.sh r4h ab:C4:ab_libs/vvo0.so,default:3 ab:C3:default,env=LDPC_BS_INST=8:2 ab:C5:ab_libs/vvo0.so,default:2 || exit 1
