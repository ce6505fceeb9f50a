# lane / LDS group-by parity tests + filter + GROUP BY SUM timings at 1B docs (quick iteration)
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lane.py -x -q --timeout 120 --timeout-method thread > $out/lane_tests.log 2>&1 || { echo tests_failed; tail -40 $out/lane_tests.log; exit 1; }
tail -2 $out/lane_tests.log
bash tools/g_sg.sh $tag
