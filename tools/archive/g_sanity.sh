# Final-tree sanity: smoke, the dense / lane parity tests, the bench line
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke_failed; cat $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_lane.py tests/test_gpu_stats.py tests/test_gpu_mv.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_failed; tail -30 $out/tests.log; exit 2; }
tail -1 $out/tests.log
timeout -k 10 300 python -u bench.py > $out/bench.json 2> $out/bench.err || { echo bench_failed; tail -20 $out/bench.err; exit 3; }
python3 -c "import json; d=json.loads(open('$out/bench.json').readline()); print(d['value'], d['roofline']['frac'], [round(x['roofline']['frac'],3) for x in d['secondary']])"
echo all_ok
