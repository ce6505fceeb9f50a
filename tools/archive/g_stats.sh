# Fused execution statistics (PA_QF_FILTER_STATS): parity tests, then configs[1] (100 segments x 10M docs) and
# configs[0] 10 % with the statistics timed against the plain scan
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stats.py -x -v --timeout 300 --timeout-method thread > $out/stats_tests.log 2>&1 || { echo tests_failed; tail -40 $out/stats_tests.log; exit 1; }
tail -2 $out/stats_tests.log
timeout -k 10 400 python -u tools/bench_configs.py --workload adanalytics --segments 100 --no-stepmajor --exec-stats > $out/adanalytics.json 2> $out/adanalytics.err || { echo bench_failed; tail -20 $out/adanalytics.err; exit 3; }
timeout -k 10 400 python -u tools/bench_configs.py --workload sumscan --plan sel_10pct --segments 100 --no-stepmajor --exec-stats > $out/sumscan.json 2> $out/sumscan.err || { echo bench_failed; tail -20 $out/sumscan.err; exit 3; }
cat $out/adanalytics.json $out/sumscan.json | python -c "import json,sys; [print(d['workload'], d['plan_name'], d['kernel_ms'], d['exec_stats']) for d in map(json.loads, sys.stdin)]"
echo all_ok
