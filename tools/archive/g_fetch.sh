# GPU parity tests + configs[2]/[4] lines (fetch timing)
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo tests_failed; tail -30 $out/gpu_tests.log; exit 1; }
tail -3 $out/gpu_tests.log
timeout -k 10 400 python -u tools/bench_configs.py --workload all --no-stepmajor > $out/configs.json 2> $out/configs.err || { echo configs_failed; tail -20 $out/configs.err; exit 5; }
cut -c1-200 $out/configs.json
echo all_ok
