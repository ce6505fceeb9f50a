# Round 6: numGroupsLimit walk replayed from registers: the limit GPU tests, then configs[2] / configs[4] lines with
# per-kernel durations (limit_walk_kernel's average is the number to compare: 0.559 ms before)
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_mv.py -k "limit or config" > $out/tests.log 2>&1 || { echo tests_failed; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for w in highcard star; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/${w}_trace -o run --output-format csv -- python3 tools/bench_configs.py --workload $w --segments 20 --no-stepmajor --reps 10 > $out/${w}.jsonl 2> $out/${w}.err || { echo ${w}_failed; tail -5 $out/${w}.err; exit 1; }
  python3 -c "
import json
for l in open('$out/${w}.jsonl'):
    d=json.loads(l); print('$w', d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'],3), d['groups'])"
  f=$(find $out/${w}_trace -name "*kernel_stats.csv" | head -1); cp $f $out/${w}_kernel_stats.csv
  grep -i walk $out/${w}_kernel_stats.csv || true
done
echo all_ok
