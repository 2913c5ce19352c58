# round 4, session m: the opaque lane index of the one-chunk instances' table copies (C2
# spill-free): whole suite, A/B against the evidence build, then the round-end evidence of this
# build (kept only if the A/B favours it)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4m; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; grep -E "FAILED|^ERROR" $O/pytest_gpu.log | head -30
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_session.sh r4m ab:C2:ab_libs/evid.so,default:3 ab:C3:ab_libs/evid.so,default:2 || exit 1
SKIP_TESTS=1 TAG=r4g bash tools/gpu_final_a.sh || exit 1
