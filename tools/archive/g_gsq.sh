# SQ counters of the dense GROUP BY kernel for a few PA_DEBUG_EMIT knobs (measurement only)
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
for d in 0 6; do
  PA_DEBUG_EMIT=$d timeout -k 10 300 bash tools/prof_cfg_sq.sh ${tag}_d$d --workload sumgroup_dict --plan sel_50pct --segments 20 --no-stepmajor --reps 3 || { echo failed_$d; exit 1; }
  python3 tools/pmc_by_kernel.py gpurun_out/prof_${tag}_d$d > $out/sq_d$d.json || exit 2
  python3 -c "
import json; d=json.load(open('$out/sq_d$d.json'))
for k,v in d.items():
    if 'gdense' in k: print($d, k[:40], {c: v[c] for c in v if c.startswith(('SQ_INSTS','SQ_WAVE_CYCLES','SQ_WAVES','frac','SQ_LDS'))})"
done
echo all_ok
