# configs[0] lines at 1B rows (100 x 10M docs) with roofline + the C-port CPU baseline (16 host segments)
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for w in sumscan sumscan_raw; do
timeout -k 10 500 python -u tools/bench_configs.py --workload $w --segments 100 --no-stepmajor --cpu-sample 16 >> $out/configs0_1b.json 2>> $out/configs0_1b.err || { echo fail; tail -5 $out/configs0_1b.err; exit 1; }
done
python3 -c "
import json
for l in open('$out/configs0_1b.json'): d=json.loads(l); print(d['workload'], d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'],3), d['cpu_baseline']['value'])
"
