# Round 5: count-free partitioned emit — parity (configs[2] tests, partitioned parity) and configs[2] timings
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -k "configs2" -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_failed; grep -E "FAILED|Error|assert" $out/tests.log | head -30; tail -5 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python -u tools/bench_configs.py --workload highcard --segments 20 --no-stepmajor --reps 10 > $out/highcard.json 2> $out/highcard.err || { echo bench_failed; tail -20 $out/highcard.err; exit 2; }
python3 -c "
import json
for l in open('$out/highcard.json'):
    d=json.loads(l); print(d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'],3), d['plan'].get('count_free_emit'), d['groups'])"
A="--workload highcard --plan all_docs --segments 20 --no-stepmajor --reps 10"
bash tools/prof_cfg.sh ${tag}_hc $A || exit 3
python3 -c "import csv,glob; r=[x for f in glob.glob('gpurun_out/prof_${tag}_hc/trace/**/*kernel_stats.csv', recursive=True) for x in csv.DictReader(open(f))]; [print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e3,1), 'us') for x in r[:8]]"
echo all_ok
