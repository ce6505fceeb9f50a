# Round 6 GPU step: the given pytest selection (-m gpu), then optionally the bench (BENCH=1) with its JSON summary.
# usage: bash tools/g_r06.sh TAG [pytest args...]
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
if [ $# -gt 0 ]; then
  timeout -k 10 1000 python -u -m pytest "$@" -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR|Error|passed|failed" $out/gpu_tests.log | tail -40
  [ $rc -ne 0 ] && { echo tests_rc=$rc; exit 1; }
fi
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > $out/bench.json 2> $out/bench.err || { echo bench_failed; tail -20 $out/bench.err; exit 3; }
  python3 -c "
import json; d=json.loads(open('$out/bench.json').readline())
print('headline', d['value'], d['roofline']['kernel_ms'], round(d['roofline']['frac'],3))
for x in d['secondary']: print(x['workload'], round(x['kernel_ms'],4), round(x['roofline']['frac'],3), x['roofline']['plan'].get('variant'), x['roofline']['plan'].get('dense_packed'), x.get('checked'), x.get('check_plan'))
"
fi
echo all_ok
