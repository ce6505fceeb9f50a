# SQ counters of the partitioned path's kernels (configs[2] all docs; measurement only)
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 bash tools/prof_cfg_sq.sh ${tag}_hc --workload highcard --plan all_docs --segments 20 --reps 3 || { echo failed; exit 1; }
python3 tools/pmc_by_kernel.py gpurun_out/prof_${tag}_hc > $out/sq_hc.json || exit 2
python3 -c "
import json; d=json.load(open('$out/sq_hc.json'))
for k,v in d.items(): print(k[:60], {c: v[c] for c in v if c.startswith(('SQ_','frac'))})"
echo all_ok
