# Round-4 final, part A: every GPU parity test, smoke, the bench line and its rocprof kernel stats
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=20 -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo tests_failed; tail -30 $out/gpu_tests.log; exit 1; }
tail -2 $out/gpu_tests.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke_failed; cat $out/smoke.log; exit 2; }
tail -2 $out/smoke.log
timeout -k 10 300 python -u bench.py > $out/bench.json 2> $out/bench.err || { echo bench_failed; tail -20 $out/bench.err; exit 3; }
cat $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 bench.py --cpu-sample 0 > $out/bench_prof.json 2> $out/bench_prof.err || { echo prof_failed; exit 4; }
python3 -c "import csv,glob; r=[x for f in glob.glob('$out/trace/**/*kernel_stats.csv', recursive=True) for x in csv.DictReader(open(f))]; [print(x['Name'][:70], x['Calls'], round(float(x['AverageNs'])/1e3,1), 'us') for x in r[:8]]"
echo all_ok
