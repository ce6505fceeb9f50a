# filter + GROUP BY SUM at 1B docs (raw and dictionary LONG metric), kernel trace for the rocprof average
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in sumgroup sumgroup_dict; do
timeout -k 10 400 python3 tools/bench_configs.py --workload $w --segments 100 --reps 10 --no-stepmajor >> $out/sg.json 2>> $out/sg.err || { echo bench_failed; tail -5 $out/sg.err; exit 1; }
done
python3 -c "
import json
for l in open('$out/sg.json'): d=json.loads(l); print(d['workload'], d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'],3), d['plan']['strategy'], d['plan']['lane_major'], d['plan']['wg_per_cu'], d['groups'])
"
