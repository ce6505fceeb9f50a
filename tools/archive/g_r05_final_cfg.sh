# Round 5 final: every configs[2] / configs[4] line (kernel trace) and the HBM bytes of both all-docs lines
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in highcard star; do
  bash tools/prof_cfg.sh ${tag}_$w --workload $w --segments 20 --no-stepmajor --reps 10 || { echo "$w failed"; tail -5 gpurun_out/prof_${tag}_$w/err.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/prof_${tag}_$w/out.json'):
    d=json.loads(l); print('$w', d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'],3), d['plan'].get('count_free_emit'))"
done
for w in highcard star; do
  bash tools/prof_cfg_hbm.sh ${tag}_hbm_$w --workload $w --plan all_docs --segments 10 --no-stepmajor --reps 2 || { echo "hbm $w failed"; exit 2; }
  python3 tools/pmc_by_kernel.py gpurun_out/prof_${tag}_hbm_$w > gpurun_out/prof_${tag}_hbm_$w/pmc.json
done
echo all_ok
