# all GPU parity tests + configs[0] at 1B docs
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo tests_failed; tail -40 $out/gpu_tests.log; exit 1; }
tail -3 $out/gpu_tests.log
bash tools/g_ss100.sh $tag
