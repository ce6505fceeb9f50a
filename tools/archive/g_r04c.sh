# Round-4 partitioned/MV/statistics check: parity tests, then configs[2] / configs[4] / mvgroup per-kernel times, the
# fused statistics at configs[1], and SQ counters of the MV emit pass
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_mv.py tests/test_gpu_parity.py tests/test_gpu_stats.py tests/test_gpu_dense.py tests/test_gpu_configs.py -k "mv or partitioned or stats or dense or configs2 or configs4" -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_failed; tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
bash tools/g_configs.sh ${tag}_hc --workload highcard --plan all_docs --segments 20 || exit 2
bash tools/g_configs.sh ${tag}_st --workload star --plan all_docs --segments 20 || exit 3
bash tools/g_configs.sh ${tag}_mv --workload mvgroup --segments 20 || exit 4
timeout -k 10 400 python -u tools/bench_configs.py --workload adanalytics --segments 100 --no-stepmajor --exec-stats > $out/adanalytics.json 2> $out/adanalytics.err || { echo bench_failed; tail -20 $out/adanalytics.err; exit 5; }
python -c "import json; d=json.loads(open('$out/adanalytics.json').readline()); print(d['kernel_ms'], d['exec_stats'])"
timeout -k 10 300 bash tools/prof_cfg_sq.sh ${tag}_mvsq --workload mvgroup --plan untrimmed --segments 20 --reps 3 || { echo sq_failed; exit 6; }
python3 tools/pmc_by_kernel.py gpurun_out/prof_${tag}_mvsq > $out/sq_mv.json || exit 7
python3 -c "
import json; d=json.load(open('$out/sq_mv.json'))
for k,v in d.items():
    if 'scan_kernel' in k or 'part_agg' in k: print(k[:40], {c: v[c] for c in v if c.startswith(('SQ_INSTS','SQ_WAVE','frac','SQ_LDS'))})"
echo all_ok
