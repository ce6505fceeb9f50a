# Round 6: the walk replay's first-lane table (PA_WALK_TAB): the limit tests, then the default-limit lines A/B
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_mv.py -k "limit or config or star" > $out/tests.log 2>&1 || { echo tests_failed; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for w in highcard star; do
for s in tab:1 notab:0; do
  n=${s%%:*}; v=${s##*:}
  PA_WALK_TAB=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/${w}_${n}_trace -o run --output-format csv -- python3 tools/bench_configs.py --workload $w --segments 20 --no-stepmajor --reps 10 --plan default_limit > $out/${w}_${n}.jsonl 2> $out/${w}_${n}.err || { echo ${n}_failed; tail -5 $out/${w}_${n}.err; exit 1; }
  python3 -c "
import json
for l in open('$out/${w}_${n}.jsonl'):
    d=json.loads(l); print('$w $n', d['plan_name'], d['kernel_ms'], d['groups'])"
  f=$(find $out/${w}_${n}_trace -name "*kernel_stats.csv" | head -1); cp $f $out/${w}_${n}_kernel_stats.csv
  grep "limit_walk" $out/${w}_${n}_kernel_stats.csv | cut -c1-150
done
done
echo all_ok
