# Round 6: configs[2] (shared and own dictionaries) and configs[4] lines timed warm (20 untimed scans, 50 timed), then
# one rocprof pass per workload for the per-kernel durations
set -o pipefail
out=gpurun_out/r06_cfgwarm
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in highcard highcard_own star; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/${w}_trace -o run --output-format csv -- python3 tools/bench_configs.py --workload $w --segments 20 --no-stepmajor --warm 20 --reps 50 > $out/${w}.jsonl 2> $out/${w}.err || { echo ${w}_failed; tail -5 $out/${w}.err; exit 1; }
  python3 -c "
import json
for l in open('$out/${w}.jsonl'):
    d=json.loads(l); print('$w', d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'],3), d['plan'].get('count_free_emit'), d['groups'])"
  f=$(find $out/${w}_trace -name "*kernel_stats.csv" | head -1); cp $f $out/${w}_kernel_stats.csv
done
echo all_ok
