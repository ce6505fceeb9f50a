# lane-path parity + configs[0] at 1B docs
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/lane_tests.log 2>&1 || { echo tests_failed; tail -40 $out/lane_tests.log; exit 1; }
tail -3 $out/lane_tests.log
bash tools/g_ss100.sh $tag
