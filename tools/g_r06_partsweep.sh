# Round 6: configs[2] / configs[4] all-docs lines over LDS per partition x workgroups per CU (PA_QF_PART / PA_QF_WG), warm
set -o pipefail
out=gpurun_out/r06_partsweep
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in highcard star; do
  timeout -k 10 300 python3 tools/bench_configs.py --workload $w --segments 20 --plan all_docs --sweep-part --warm 20 --reps 30 > $out/${w}.jsonl 2> $out/${w}.err || { echo ${w}_failed; tail -5 $out/${w}.err; exit 1; }
  python3 -c "
import json
for l in open('$out/${w}.jsonl'):
    d=json.loads(l); p=d['plan']; print('$w', d['plan_name'], d['kernel_ms'], d['groups'], p.get('count_free_emit'), p.get('grid'), p.get('lds_bytes'), p.get('wg_per_cu'))"
done
echo all_ok
