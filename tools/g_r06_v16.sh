# Round 6: pass C's V partitions at 16 waves per workgroup, one register batch (PA_PASSC_V16=1): partitioned-path
# parity tests with it on, then configs[2] / configs[4] A/B with per-kernel durations
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PA_PASSC_V16=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mv.py tests/test_gpu_configs.py tests/test_gpu_parity.py -k "star or partitioned or config or limit or hll" > $out/tests.log 2>&1 || { echo tests_failed; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for w in highcard star; do
for s in v16:1 v8:0 v16b:1; do
  n=${s%%:*}; v=${s##*:}
  PA_PASSC_V16=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/${w}_${n}_trace -o run --output-format csv -- python3 tools/bench_configs.py --workload $w --segments 20 --no-stepmajor --reps 10 > $out/${w}_${n}.jsonl 2> $out/${w}_${n}.err || { echo ${n}_failed; tail -5 $out/${w}_${n}.err; exit 1; }
  python3 -c "
import json
for l in open('$out/${w}_${n}.jsonl'):
    d=json.loads(l); print('$w $n', d['plan_name'], d['kernel_ms'], d['groups'])"
  f=$(find $out/${w}_${n}_trace -name "*kernel_stats.csv" | head -1); cp $f $out/${w}_${n}_kernel_stats.csv
  grep "part_agg" $out/${w}_${n}_kernel_stats.csv | cut -c1-150
done
done
echo all_ok
