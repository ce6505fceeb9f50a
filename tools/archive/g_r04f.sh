# Dense GROUP BY with more accumulator replicas: parity tests + the configs[0]/configs[1]-shape lines
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_lane.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_failed; tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for w in sumgroup_dict adanalytics_in sumgroup; do
  timeout -k 10 400 python -u tools/bench_configs.py --workload $w --segments 100 --no-stepmajor > $out/configs_$w.json 2> $out/configs_$w.err || { echo configs_failed $w; tail -20 $out/configs_$w.err; exit 2; }
  python3 -c "import json; [print(d['workload'], d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'], 3), d['plan']['strategy'], d['plan']['lds_bytes']) for d in map(json.loads, open('$out/configs_$w.json'))]"
done
echo all_ok
