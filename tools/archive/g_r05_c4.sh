# Round 5: configs[4] count-free emit (both streams): its parity tests, then the star line's kernel profile
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_mv.py -k "configs4 or star or partitioned" -x -v --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_failed; grep -E "FAILED|Error|assert|Mismatch" $out/tests.log | head -30; tail -5 $out/tests.log; exit 1; }
tail -2 $out/tests.log
PA_DEBUG_PLAN=1 bash tools/prof_cfg.sh ${tag}_star --workload star --plan all_docs --segments 20 --no-stepmajor --reps 10 || { echo prof_failed; tail -5 gpurun_out/prof_${tag}_star/err.log; exit 2; }
python3 -c "import csv,glob; r=[x for f in glob.glob('gpurun_out/prof_${tag}_star/trace/**/*kernel_stats.csv', recursive=True) for x in csv.DictReader(open(f))]; [print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e3,1), 'us') for x in r[:8]]"
grep -E "pve" gpurun_out/prof_${tag}_star/err.log | head -4
head -c 600 gpurun_out/prof_${tag}_star/out.json
echo all_ok
