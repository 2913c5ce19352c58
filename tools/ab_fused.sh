set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_v3.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_v3.log; [ $rc -ne 0 ] && exit $rc
for v in 2 3; do LDPC_FUSED_VERSION=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_v$v.json || exit 1; python -c "import json;d=json.load(open('gpurun_out/bench_v$v.json'));print('v$v', d['value'], d['config']['kernel'], d['ms_per_step'])"; done
