# Round 6: every GPU parity test, smoke, the bench line, its rocprof kernel stats and the launcher (world size 1) line
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=20 -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo tests_failed; grep -E "FAILED|Error" $out/gpu_tests.log | head -30; tail -3 $out/gpu_tests.log; exit 1; }
tail -2 $out/gpu_tests.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke_failed; cat $out/smoke.log; exit 2; }
tail -2 $out/smoke.log
timeout -k 10 300 python -u bench.py > $out/bench.json 2> $out/bench.err || { echo bench_failed; tail -20 $out/bench.err; exit 3; }
python3 -c "
import json; d=json.loads(open('$out/bench.json').readline())
print('headline', d['value'], d['roofline']['kernel_ms'], round(d['roofline']['frac'],3), d['cpu_baseline'])
for x in d['secondary']: print(x['workload'], x['kernel_ms'], round(x['roofline']['frac'],3), x['roofline']['plan'].get('variant'), x['roofline']['plan'].get('dense_packed'))
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 bench.py --cpu-sample 0 > $out/bench_prof.json 2> $out/bench_prof.err || { echo prof_failed; exit 4; }
python3 -c "import csv,glob; r=[x for f in glob.glob('$out/trace/**/*kernel_stats.csv', recursive=True) for x in csv.DictReader(open(f))]; [print(x['Name'][:70], x['Calls'], round(float(x['AverageNs'])/1e3,1), 'us') for x in r[:8]]"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-secondary > $out/bench_launcher.json 2> $out/bench_launcher.err || { echo launcher_failed; tail -20 $out/bench_launcher.err; exit 5; }
python3 -c "import json; d=json.loads(open('$out/bench_launcher.json').readline()); print('launcher', d['value'], d.get('multi_gpu'))"
echo all_ok
