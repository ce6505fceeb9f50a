# Lane-path parity (aggregation-only: raw / dictionary, sparse / dense tiles) + configs[0] timings at 200M docs
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/lane_tests.log 2>&1 || { echo tests_failed; tail -40 $out/lane_tests.log; exit 1; }
tail -3 $out/lane_tests.log
for w in sumscan sumscan_raw; do
timeout -k 10 300 python -u tools/bench_configs.py --workload $w --segments 20 --no-stepmajor >> $out/ss.json 2>> $out/ss.err || { echo bench_failed; tail -20 $out/ss.err; exit 2; }
done
python3 -c "
import json
for l in open('$out/ss.json'): d=json.loads(l); print(d['workload'], d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'],3) if 'roofline' in d else '')
"
