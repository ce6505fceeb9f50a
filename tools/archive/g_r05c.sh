# Round 5: lane-major dense GROUP BY walk (STRAT_GDENSE_LM*): dense parity tests, configs[1] lines, bench secondary lines
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_configs.py -k "dense or configs1 or configs0" -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_failed; tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
for w in adanalytics_in sumgroup_dict sumgroup; do
  timeout -k 10 400 python -u tools/bench_configs.py --workload $w --segments 100 --no-stepmajor > $out/configs_$w.json 2> $out/configs_$w.err || { echo configs_failed $w; tail -20 $out/configs_$w.err; exit 2; }
  python3 -c "import json; [print(d['workload'], d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'], 3), d['plan']['strategy'], d['plan'].get('variant'), d['plan']['wg_per_cu'], d['plan']['lds_bytes']) for d in map(json.loads, open('$out/configs_$w.json'))]"
done
echo all_ok
