# PA_QF_LAZY_POST across the configs workloads at <= 50 % filter density (200M docs)
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for wp in "highcard filtered_10pct" "sumscan sel_10pct" "sumscan sel_50pct" "sumscan sel_1pct" "sumscan_raw sel_10pct" "sumscan_raw sel_50pct"; do
set -- $wp
for f in 0 268435456; do
timeout -k 10 200 python3 tools/bench_configs.py --workload $1 --plan $2 --segments 20 --reps 10 --flags $f >> $out/lp.json 2>> $out/lp.err || { echo bench_failed; tail -5 $out/lp.err; exit 1; }
done
done
python3 -c "
import json
for l in open('$out/lp.json'): d=json.loads(l); print(d['workload'], d['plan_name'], d['kernel_ms'], d['plan']['strategy'], d['plan']['wg_per_cu'], d['plan']['ring'])
"
