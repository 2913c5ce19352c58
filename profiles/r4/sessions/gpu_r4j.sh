# round 4, session j: bsc without the per-chunk alpha-table register (recomputed per use)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bitsliced.py tests/test_gpu_periter.py tests/test_gpu_channel.py -m gpu -v -rs --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; grep -E "FAILED|^ERROR" $O/pytest_gpu.log | head -30
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_session.sh r4j ab:C5:ab_libs/pre_gtab.so,default:3 || exit 1
