# round 4, last session: the driver's round-end sequence on the final tree (pytest -m gpu,
# smoke, the default bench line)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4z; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
