# MV group-by on the partitioned path: parity tests (MV + partitioned), then mvgroup untrimmed / default limit timings
# and a kernel trace of the untrimmed plan
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_mv.py tests/test_gpu_parity.py -k "mv or partitioned" -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_failed; tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python3 tools/bench_configs.py --workload mvgroup --segments 20 --no-stepmajor > $out/mv.json 2> $out/mv.err || { echo bench_failed; tail -5 $out/mv.err; exit 1; }
python3 -c "
import json
for l in open('$out/mv.json'): d=json.loads(l); print(d['plan_name'], d['kernel_ms'], d['fetch_ms'], d['groups'], d['plan']['strategy'], d['plan']['limit_trimming'])
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt -o run --output-format csv -- python3 tools/bench_configs.py --workload mvgroup --plan untrimmed --segments 20 --reps 3 --no-stepmajor > /dev/null 2> $out/kt.err || { echo kt_failed; exit 2; }
python3 -c "
import csv,glob
for f in glob.glob('$out/kt/**/*kernel_stats.csv', recursive=True):
    for r in list(csv.DictReader(open(f)))[:12]: print('  ', r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
echo all_ok
