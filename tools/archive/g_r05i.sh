# Round 5: dense parity tests + bench (secondary lines on the query-shape specialised kernel)
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_configs.py -k "dense or configs1 or configs0" -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_failed; tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-sample 0 > $out/bench.json 2> $out/bench.err || { echo bench_failed; tail -20 $out/bench.err; exit 2; }
python3 -c "
import json; d=json.loads(open('$out/bench.json').readline())
print('headline', d['value'], d['roofline']['kernel_ms'], round(d['roofline']['frac'],3))
for x in d['secondary']: print(x['workload'], x['kernel_ms'], round(x['roofline']['frac'],3), x['roofline']['plan'].get('variant'), x['roofline']['plan'].get('dense_packed'))
"
echo all_ok
