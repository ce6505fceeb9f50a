# Round 5: configs[4] HBM read / write bytes per kernel, count-free emit vs count + emit passes
set -o pipefail
tag=$1
A="--workload star --plan all_docs --segments 10 --no-stepmajor --reps 2"
bash tools/prof_cfg_hbm.sh ${tag}_base $A || { echo base_failed; exit 1; }
PA_NO_JIT=1 bash tools/prof_cfg_hbm.sh ${tag}_old $A || { echo old_failed; exit 2; }
for n in base old; do python3 tools/pmc_by_kernel.py gpurun_out/prof_${tag}_$n > gpurun_out/prof_${tag}_$n/pmc.json; python3 -c "
import json; d=json.load(open('gpurun_out/prof_${tag}_$n/pmc.json'))
for k,v in d.items():
  if any(s in k for s in ('pve_jit','part_agg','scan_kernel')): print('$n', k[:40], {a: round(b,1) for a,b in v.items() if a in ('hbm_read_MB','hbm_write_MB','dispatches')})
"; done
echo all_ok
