# Multi-rank merge paths on one GPU (RCCL world size 1 + simulated ranks): tests/test_gpu_dist.py
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 200 --timeout-method thread > $out/dist_tests.log 2>&1 || { echo tests_failed; tail -40 $out/dist_tests.log; exit 1; }
tail -2 $out/dist_tests.log
echo all_ok
