# Round 5: configs[2] partitioned kernels decomposition (per-kernel rocprof averages): full, emit bins dropped
# (PA_DEBUG_EMIT=1), stream only (PA_QF_DEBUG_STREAM_ONLY)
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A="--workload highcard --plan all_docs --segments 20 --no-stepmajor --reps 10"
bash tools/prof_cfg.sh ${tag}_full $A || exit 1
PA_DEBUG_EMIT=1 bash tools/prof_cfg.sh ${tag}_drop $A || exit 2
bash tools/prof_cfg.sh ${tag}_stream $A --flags 65536 || exit 3
for v in full drop stream; do
python3 -c "import csv,glob; r=[x for f in glob.glob('gpurun_out/prof_${tag}_$v/trace/**/*kernel_stats.csv', recursive=True) for x in csv.DictReader(open(f))]; [print('$v', x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e3,1), 'us') for x in r if 'scan_kernel' in x['Name'] or 'part_' in x['Name']]"
done
echo all_ok
