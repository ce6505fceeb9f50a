# Round 6: pass C's H partitions in their own 16-wave launch: H-stream parity tests, then configs[4] A/B
# (PA_PASSC_H_SPLIT=0: H partitions inside the 8-wave V launch) with per-kernel durations
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mv.py tests/test_gpu_configs.py tests/test_gpu_parity.py -k "star or partitioned or configs4 or hll" > $out/tests.log 2>&1 || { echo tests_failed; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for s in split:1 nosplit:0 split2:1; do
  n=${s%%:*}; v=${s##*:}
  PA_PASSC_H_SPLIT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/star_${n}_trace -o run --output-format csv -- python3 tools/bench_configs.py --workload star --segments 20 --no-stepmajor --reps 10 > $out/star_${n}.jsonl 2> $out/star_${n}.err || { echo ${n}_failed; tail -5 $out/star_${n}.err; exit 1; }
  python3 -c "
import json
for l in open('$out/star_${n}.jsonl'):
    d=json.loads(l); print('$n', d['plan_name'], d['kernel_ms'], d['groups'])"
  f=$(find $out/star_${n}_trace -name "*kernel_stats.csv" | head -1); cp $f $out/star_${n}_kernel_stats.csv
  grep "part_agg" $out/star_${n}_kernel_stats.csv | cut -c1-150
done
echo all_ok
