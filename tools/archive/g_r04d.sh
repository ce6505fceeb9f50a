# Round-4 check: fused statistics (tests, configs[1] / configs[0] 10 % timings, kernel trace) + partitioned lines
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_mv.py tests/test_gpu_parity.py tests/test_gpu_configs.py -k "mv or partitioned or configs2 or configs4" -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_failed; tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
bash tools/g_stats.sh ${tag}_s || exit 2
bash tools/g_stats_prof.sh ${tag}_sp || exit 3
bash tools/g_configs.sh ${tag}_hc --workload highcard --plan all_docs --segments 20 || exit 4
bash tools/g_configs.sh ${tag}_st --workload star --plan all_docs --segments 20 || exit 5
bash tools/g_configs.sh ${tag}_mv --workload mvgroup --segments 20 || exit 6
echo all_ok
