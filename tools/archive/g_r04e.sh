# Dense GROUP BY after the RS12 spill fix + fused statistics search: parity tests, 1B-doc lines, decomposition
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_stats.py tests/test_gpu_lane.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_failed; tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for w in sumgroup_dict adanalytics_in sumgroup; do
  timeout -k 10 400 python -u tools/bench_configs.py --workload $w --segments 100 --no-stepmajor > $out/configs_$w.json 2> $out/configs_$w.err || { echo configs_failed $w; tail -20 $out/configs_$w.err; exit 2; }
  python3 -c "import json; [print(d['workload'], d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'], 3), d['plan']['strategy'], d['plan']['dma_slots']) for d in map(json.loads, open('$out/configs_$w.json'))]"
done
timeout -k 10 400 python -u tools/bench_configs.py --workload adanalytics --segments 100 --no-stepmajor --exec-stats > $out/exec_stats_adanalytics.json 2> $out/exec_stats.err || { echo stats_failed; tail -20 $out/exec_stats.err; exit 3; }
python3 -c "import json; d=json.loads(open('$out/exec_stats_adanalytics.json').readline()); print(d['kernel_ms'], d['exec_stats'])"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/stats_trace -o run --output-format csv -- python3 tools/bench_configs.py --workload adanalytics --segments 100 --reps 10 --no-stepmajor --exec-stats > /dev/null 2> $out/stats_trace.err || { echo stats_prof_failed; exit 4; }
python3 -c "import csv,glob; r=[x for f in glob.glob('$out/stats_trace/**/*kernel_stats.csv', recursive=True) for x in csv.DictReader(open(f))]; [print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e3,1), 'us') for x in r if 'leap' in x['Name'] or 'scan_kernel' in x['Name']]"
bash tools/g_gdbg2.sh ${tag}_gd || exit 5
echo all_ok
