# filter + GROUP BY SUM at 1B docs: post-filter columns staged (auto) vs read per matching doc (PA_QF_LAZY_POST)
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in sumgroup_dict sumgroup; do
for f in 0 268435456; do
timeout -k 10 300 python3 tools/bench_configs.py --workload $w --segments 100 --reps 10 --flags $f >> $out/lp.json 2>> $out/lp.err || { echo bench_failed; tail -5 $out/lp.err; exit 1; }
done
done
python3 -c "
import json
for l in open('$out/lp.json'): d=json.loads(l); print(d['workload'], d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'],3), d['plan']['strategy'], d['plan']['wg_per_cu'], d['plan']['ring'])
"
