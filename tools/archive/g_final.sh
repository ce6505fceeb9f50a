# Round-end check on the GPU box: parity tests, smoke, bench line, rocprof kernel stats, configs[2]/[4] lines
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo tests_failed; tail -30 $out/gpu_tests.log; exit 1; }
tail -3 $out/gpu_tests.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke_failed; cat $out/smoke.log; exit 2; }
cat $out/smoke.log
timeout -k 10 300 python -u bench.py > $out/bench.json 2> $out/bench.err || { echo bench_failed; tail -20 $out/bench.err; exit 3; }
cat $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 bench.py --cpu-sample 0 > $out/bench_prof.json 2> $out/bench_prof.err || { echo prof_failed; exit 4; }
timeout -k 10 400 python -u tools/bench_configs.py --workload all > $out/configs.json 2> $out/configs.err || { echo configs_failed; tail -20 $out/configs.err; exit 5; }
cat $out/configs.json
echo all_ok
