# configs[0] (sumscan / sumscan_raw) timings at 1B docs (100 segments), 20 reps per plan
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for w in sumscan sumscan_raw; do
timeout -k 10 400 python -u tools/bench_configs.py --workload $w --segments 100 --reps 20 --no-stepmajor >> $out/ss100.json 2>> $out/ss100.err || { echo bench_failed; tail -20 $out/ss100.err; exit 2; }
done
python3 -c "
import json
for l in open('$out/ss100.json'): d=json.loads(l); print(d['workload'], d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'],3), d['plan']['ring'], d['plan']['wg_per_cu'])
"
