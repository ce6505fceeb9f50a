# execution statistics on the GPU: parity (pa_bitmap_counts vs numpy, device closed forms vs host replay, golden
# statistics) + cost at configs[1] scale (100 x 10M-doc AdAnalytics segments) and on configs[0]'s shape
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stats.py "tests/test_gpu_parity.py::test_golden_cases_gpu" -x -v --timeout 300 --timeout-method thread > $out/stats_tests.log 2>&1 || { echo tests_failed; tail -40 $out/stats_tests.log; exit 1; }
tail -3 $out/stats_tests.log
timeout -k 10 500 python3 tools/bench_configs.py --workload adanalytics --segments 100 --reps 10 --no-stepmajor --exec-stats > $out/stats.json 2> $out/stats.err || { echo bench_failed; tail -5 $out/stats.err; exit 1; }
timeout -k 10 300 python3 tools/bench_configs.py --workload sumscan --plan sel_10pct --segments 100 --reps 10 --no-stepmajor --exec-stats >> $out/stats.json 2>> $out/stats.err || { echo bench_failed; tail -5 $out/stats.err; exit 1; }
python3 -c "
import json
for l in open('$out/stats.json'): d=json.loads(l); print(d['workload'], d['plan_name'], d['kernel_ms'], d['exec_stats'])
"
