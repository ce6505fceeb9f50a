# Round 6: the MV walk replay's first-lane table: MV / limit GPU tests, then the mvgroup default-limit line A/B
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mv.py tests/test_gpu_parity.py -k "limit or walk or mv" > $out/tests.log 2>&1 || { echo tests_failed; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for s in tab:1 notab:0; do
  n=${s%%:*}; v=${s##*:}
  PA_WALK_TAB=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/mv_${n}_trace -o run --output-format csv -- python3 tools/bench_configs.py --workload mvgroup --segments 20 --no-stepmajor --reps 10 > $out/mv_${n}.jsonl 2> $out/mv_${n}.err || { echo ${n}_failed; tail -5 $out/mv_${n}.err; exit 1; }
  python3 -c "
import json
for l in open('$out/mv_${n}.jsonl'):
    d=json.loads(l); print('mv $n', d['plan_name'], d['kernel_ms'], d['groups'])"
  f=$(find $out/mv_${n}_trace -name "*kernel_stats.csv" | head -1); cp $f $out/mv_${n}_kernel_stats.csv
  grep "limit_walk" $out/mv_${n}_kernel_stats.csv | cut -c1-150 || true
done
echo all_ok
