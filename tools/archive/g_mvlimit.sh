# MV group-by at the default numGroupsLimit (sorted-form first-seen trimming) vs untrimmed: timings + per-kernel trace
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 tools/bench_configs.py --workload mvgroup --segments 20 --no-stepmajor > $out/mv.json 2> $out/mv.err || { echo bench_failed; tail -5 $out/mv.err; exit 1; }
python3 -c "
import json
for l in open('$out/mv.json'): d=json.loads(l); print(d['plan_name'], d['kernel_ms'], d['fetch_ms'], d['groups'], d['plan']['strategy'], d['plan']['limit_trimming'])
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt -o run --output-format csv -- python3 tools/bench_configs.py --workload mvgroup --plan default_limit --segments 20 --reps 3 --no-stepmajor > /dev/null 2> $out/kt.err || { echo kt_failed; exit 2; }
python3 -c "
import csv,glob
for f in glob.glob('$out/kt/**/*kernel_stats.csv', recursive=True):
    for r in list(csv.DictReader(open(f)))[:12]: print('  ', r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
