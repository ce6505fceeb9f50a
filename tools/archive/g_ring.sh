# sumscan plans under forced ring depths / workgroups per CU (flags), dictionary and raw metric
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for f in 0 $((3<<8)) $((4<<8)) $((3<<8 | 2<<12)) $((4<<8 | 2<<12)) $((6<<8 | 1<<12)); do
  timeout -k 10 200 python -u tools/bench_configs.py --workload sumscan --segments 20 --flags $f >> $out/ring.json 2>> $out/ring.err || { echo fail; tail -5 $out/ring.err; exit 1; }
done
timeout -k 10 200 python -u tools/bench_configs.py --workload sumscan_raw --segments 20 --no-stepmajor >> $out/raw.json 2>> $out/raw.err || { echo fail; tail -5 $out/raw.err; exit 1; }
python3 -c "
import json
for l in open('$out/ring.json'): d=json.loads(l); print(d['plan_name'], d['kernel_ms'], round(d['staged_GBps']), d['plan']['ring'], d['plan']['wg_per_cu'])
for l in open('$out/raw.json'): d=json.loads(l); print('raw', d['plan_name'], d['kernel_ms'], round(d['staged_GBps']), d['plan'])
"
