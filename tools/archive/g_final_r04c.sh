# Round-4 final, part C: HBM traffic per kernel (PMC FETCH_SIZE / WRITE_SIZE in separate passes, gfx950 x2 read
# correction in tools/pmc_by_kernel.py) of configs[2], configs[4], the MV GROUP BY and GROUP BY day SUM(dictionary m)
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for spec in "highcard all_docs 10" "star all_docs 10" "mvgroup untrimmed 10" "sumgroup_dict sel_50pct 10" "sumgroup sel_50pct 10"; do
  set -- $spec
  bash tools/prof_cfg_hbm.sh ${tag}_$1 --workload $1 --plan $2 --segments $3 --reps 2 --no-stepmajor || { echo pmc_failed $1; exit 1; }
  python3 tools/pmc_by_kernel.py gpurun_out/prof_${tag}_$1 > $out/hbm_$1.json || exit 2
  python3 -c "
import json; d=json.load(open('$out/hbm_$1.json'))
for k,v in d.items():
    if v.get('hbm_read_MB', 0) + v.get('hbm_write_MB', 0) > 50: print('$1', k[:48], v.get('dispatches'), 'read MB', v.get('hbm_read_MB'), 'write MB', v.get('hbm_write_MB'))"
done
echo all_ok
