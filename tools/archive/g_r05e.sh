# Round 5: lane-major dense walk: decomposition of both bench secondary lines + configs lines + dense parity
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for plan in sel_10pct sel_50pct; do
for d in 32 1 2 0; do
  PA_DEBUG_EMIT=$d timeout -k 10 300 python -u tools/bench_configs.py --workload adanalytics_in --plan $plan --segments 100 --no-stepmajor > $out/${plan}_d$d.json 2> $out/${plan}_d$d.err || { echo failed_$d; tail -5 $out/${plan}_d$d.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$out/${plan}_d$d.json').readline()); print('adanalytics_in $plan', 'dbg', $d, d['kernel_ms'], round(d['roofline']['frac'],3), d['plan'].get('variant'), d['plan']['ring'], d['plan']['lds_bytes'])"
done
done
for w in sumgroup_dict sumgroup; do
  timeout -k 10 400 python -u tools/bench_configs.py --workload $w --segments 100 --no-stepmajor > $out/configs_$w.json 2> $out/configs_$w.err || { echo configs_failed $w; tail -20 $out/configs_$w.err; exit 2; }
  python3 -c "import json; [print(d['workload'], d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'], 3), d['plan'].get('variant'), d['plan']['wg_per_cu'], d['plan']['lds_bytes']) for d in map(json.loads, open('$out/configs_$w.json'))]"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_configs.py -k "dense or configs1 or configs0" -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_failed; tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
echo all_ok
