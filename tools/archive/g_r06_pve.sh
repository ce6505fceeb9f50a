# Round 6: count-free emit variants (environment knobs read at query prepare) on configs[2] / configs[4] all-docs lines
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "base:" "sent:PA_PVE_SENT=1" "pb8:PA_PVE_PB=8" "sent_pb8:PA_PVE_SENT=1 PA_PVE_PB=8"; do
  name=${v%%:*}; envs=${v#*:}
  for w in highcard star; do
    env $envs timeout -k 10 300 python -u tools/bench_configs.py --workload $w --plan all_docs --segments 20 --no-stepmajor --reps 10 > $out/${w}_$name.jsonl 2> $out/${w}_$name.err || { echo ${w}_${name}_failed; tail -5 $out/${w}_$name.err; exit 1; }
    python3 -c "
import json
for l in open('$out/${w}_$name.jsonl'):
    d=json.loads(l); print('$w', '$name', d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'],3), d['plan'].get('count_free_emit'), d['groups'])"
  done
done
echo all_ok
