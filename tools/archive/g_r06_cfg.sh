# Round 6: configs[2] lines (shared and own dictionaries) and configs[4] through tools/bench_configs.py (HIP events)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in "$@"; do
  timeout -k 10 400 python -u tools/bench_configs.py --workload $w --segments 20 --no-stepmajor --reps 10 > $out/cfg_$w.jsonl 2> $out/cfg_$w.err || { echo cfg_${w}_failed; tail -5 $out/cfg_$w.err; exit 1; }
  python3 -c "
import json
for l in open('$out/cfg_$w.jsonl'):
    d=json.loads(l); print('$w', d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'],3), d['plan'].get('count_free_emit'), d['groups'])"
done
echo all_ok
