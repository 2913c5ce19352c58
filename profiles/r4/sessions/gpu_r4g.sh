# round 4, session g: the real-edge-position word (bsl multi-chunk, bsc) and BS_KEEP_MC = 7 on
# the GPU: the whole suite, then A/B against the previous build (pre_rp) on C4 and C5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; grep -E "FAILED|^ERROR" $O/pytest_gpu.log | head -30
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_session.sh r4g ab:C4:ab_libs/pre_rp.so,ab_libs/rpw0.so,default:2 ab:C5:ab_libs/pre_rp.so,default:2 || exit 1
