# Round 5: execution statistics engine (pa_query_execution_stats) on the GPU: stats tests, golden cases, smoke, bench
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_stats.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_failed; grep -E "FAILED|Error|assert" $out/tests.log | head -30; tail -5 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-secondary > $out/bench.json 2> $out/bench.err || { echo bench_failed; tail -20 $out/bench.err; exit 2; }
python3 -c "
import json; d=json.loads(open('$out/bench.json').readline())
print('headline', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], round(d['roofline']['frac'],3), d['stats_step'])"
echo all_ok
