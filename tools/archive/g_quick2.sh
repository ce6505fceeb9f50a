# parity (all GPU tests) + configs[0] sumscan lines
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo tests_failed; tail -40 $out/gpu_tests.log; exit 1; }
tail -3 $out/gpu_tests.log
timeout -k 10 400 python -u tools/bench_configs.py --workload sumscan --segments 100 --no-stepmajor > $out/sumscan.json 2> $out/sumscan.err || { echo sumscan_failed; tail -20 $out/sumscan.err; exit 2; }
cat $out/sumscan.json
