# Round 5: count-free emit decomposition (PA_PVE_DBG: 1 records only, 2 no chunk stores; PA_PVE_PB put batch)
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A="--workload highcard --plan all_docs --segments 20 --no-stepmajor --reps 10"
for v in $VARIANTS; do
  n=${v%%:*}; e=${v#*:}
  env $e bash tools/prof_cfg.sh ${tag}_$n $A || { echo "$n failed"; tail -5 gpurun_out/prof_${tag}_$n/err.log; exit 1; }
  python3 -c "import csv,glob; r=[x for f in glob.glob('gpurun_out/prof_${tag}_$n/trace/**/*kernel_stats.csv', recursive=True) for x in csv.DictReader(open(f))]; [print('$n', x['Name'][:40], round(float(x['AverageNs'])/1e3,1), 'us') for x in r if 'pve_jit' in x['Name'] or 'part_agg' in x['Name']]"
done
echo all_ok
