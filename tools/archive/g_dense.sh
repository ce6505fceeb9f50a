# Dense GROUP BY kernel (STRAT_GDENSE): parity tests + configs[0]-shape GROUP BY lines at 1B docs
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py -x -v --timeout 120 --timeout-method thread > $out/dense_tests.log 2>&1 || { echo tests_failed; tail -40 $out/dense_tests.log; exit 1; }
tail -2 $out/dense_tests.log
for w in sumgroup_dict sumgroup adanalytics_in; do
  timeout -k 10 400 python -u tools/bench_configs.py --workload $w --segments 100 --no-stepmajor > $out/$w.json 2> $out/$w.err || { echo bench_failed $w; tail -20 $out/$w.err; exit 3; }
  cat $out/$w.json | python -c "import json,sys; [print(d['workload'], d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'],3), d['plan']['strategy'], d['plan']['ring'], d['plan']['wg_per_cu']) for d in map(json.loads, sys.stdin)]"
done
echo all_ok
