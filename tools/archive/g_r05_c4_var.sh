# Round 5: configs[4] count-free emit variants (VARIANTS="name:ENV=.. ..."): per-launch durations of both emits and pass C
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A="--workload star --plan ${PLAN:-all_docs} --segments 20 --no-stepmajor --reps 6"
for v in $VARIANTS; do
  n=${v%%:*}; e=${v#*:}
  env PA_DEBUG_PLAN=1 $e bash tools/prof_cfg.sh ${tag}_$n $A || { echo "$n failed"; tail -5 gpurun_out/prof_${tag}_$n/err.log; exit 1; }
  python3 -c "
import csv
r=list(csv.DictReader(open('gpurun_out/prof_${tag}_$n/trace/run_kernel_trace.csv')))
s=[(x['Kernel_Name'][:24], round((int(x['End_Timestamp'])-int(x['Start_Timestamp']))/1e3,1)) for x in r if 'pve_jit' in x['Kernel_Name'] or 'part_agg' in x['Kernel_Name'] or 'scan_kernel' in x['Kernel_Name']]
print('$n', s[-5:])
import json; print('$n', json.loads(open('gpurun_out/prof_${tag}_$n/out.json').readline())['kernel_ms'])
"
  grep -E "pve" gpurun_out/prof_${tag}_$n/err.log | head -2
done
echo all_ok
