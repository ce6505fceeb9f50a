# Round 5: SQ counters of the lane-major dense walk on the bench secondary plan under PA_DEBUG_EMIT modes
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for d in 65 1 32 0; do
  PA_DEBUG_EMIT=$d bash tools/prof_cfg_sq.sh ${tag}_d$d --workload adanalytics_in --plan sel_50pct --segments 20 --no-stepmajor --reps 3 || { echo prof_failed_$d; exit 1; }
  python3 tools/pmc_by_kernel.py gpurun_out/prof_${tag}_d$d > gpurun_out/prof_${tag}_d$d/summary.json
  python3 -c "
import json; d=json.load(open('gpurun_out/prof_${tag}_d$d/summary.json'))
for k,v in d.items():
    if 'gdense' in k: print($d, k[:40], {c: v.get(c) for c in ('SQ_WAVES','SQ_INSTS_VALU','SQ_INSTS_SALU','SQ_INSTS_LDS','SQ_INSTS_SMEM','SQ_LDS_BANK_CONFLICT','frac_WAIT_ANY','frac_WAIT_INST_ANY','frac_ACTIVE_INST_ANY','frac_ACTIVE_INST_VALU','frac_ACTIVE_INST_LDS','SQ_WAVE_CYCLES')})
"
done
echo all_ok
