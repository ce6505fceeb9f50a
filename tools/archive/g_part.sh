# Partitioned-path check on the GPU box: the partitioned/star/limit parity tests, then configs[2] / configs[4] lines
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "partition or star or limit or strategies or hll or golden" --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_failed; tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python -u tools/bench_configs.py --workload highcard --no-stepmajor > $out/configs.json 2> $out/configs.err || { echo hc_failed; tail -20 $out/configs.err; exit 2; }
timeout -k 10 300 python -u tools/bench_configs.py --workload star --no-stepmajor >> $out/configs.json 2>> $out/configs.err || { echo star_failed; tail -20 $out/configs.err; exit 3; }
timeout -k 10 300 python -u tools/bench_configs.py --workload highcard_rd --no-stepmajor >> $out/configs.json 2>> $out/configs.err || { echo hcrd_failed; tail -20 $out/configs.err; exit 4; }
python3 -c "
import json
for l in open('$out/configs.json'):
    d=json.loads(l); print(d['workload'], d['plan_name'], d['kernel_ms'], d['groups'], d['plan']['limit_trimming'])"
