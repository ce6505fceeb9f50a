# all GPU parity tests + configs[2]/[4] scan and fetch timings (200M docs)
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo tests_failed; tail -40 $out/gpu_tests.log; exit 1; }
tail -3 $out/gpu_tests.log
for w in highcard star; do
timeout -k 10 300 python -u tools/bench_configs.py --workload $w --segments 20 --no-stepmajor >> $out/cfg.json 2>> $out/cfg.err || { echo bench_failed; tail -20 $out/cfg.err; exit 2; }
done
python3 -c "
import json
for l in open('$out/cfg.json'): d=json.loads(l); print(d['workload'], d['plan_name'], d['kernel_ms'], d['fetch_ms'], d['e2e_ms'], d['groups'])
"
