# Round 6: the H stream's run claims (one claim per run of a doc's values): parity tests on the H stream, then the
# configs[4] line A/B (PA_PVE_HRUN=0: one claim per value; run lengths 5 / 8) with per-kernel durations; the
# numGroupsLimit walk with column-major key loads (limit tests, the default-limit lines' limit_walk_kernel)
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mv.py tests/test_gpu_configs.py tests/test_gpu_parity.py -k "star or partitioned or config or limit" > $out/tests.log 2>&1 || { echo tests_failed; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for s in run5:1:5 run8:1:8 perval:0:5 run5b:1:5; do
  n=${s%%:*}; r=$(echo $s | cut -d: -f2); b=${s##*:}
  PA_DEBUG_PLAN=1 PA_PVE_HRUN=$r PA_PVE_HB=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/star_${n}_trace -o run --output-format csv -- python3 tools/bench_configs.py --workload star --segments 20 --no-stepmajor --reps 10 --plan all_docs > $out/star_${n}.jsonl 2> $out/star_${n}.err || { echo ${n}_failed; tail -5 $out/star_${n}.err; exit 1; }
  python3 -c "
import json
for l in open('$out/star_${n}.jsonl'):
    d=json.loads(l); print('$n', d['plan_name'], d['kernel_ms'], d['groups'])"
  grep "pve H" $out/star_${n}.err | head -1
  f=$(find $out/star_${n}_trace -name "*kernel_stats.csv" | head -1); cp $f $out/star_${n}_kernel_stats.csv
  head -4 $out/star_${n}_kernel_stats.csv | cut -c1-160
done
for w in highcard star; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/${w}_dl_trace -o run --output-format csv -- python3 tools/bench_configs.py --workload $w --segments 20 --no-stepmajor --reps 10 --plan default_limit > $out/${w}_dl.jsonl 2> $out/${w}_dl.err || { echo ${w}_dl_failed; tail -5 $out/${w}_dl.err; exit 1; }
  python3 -c "
import json
for l in open('$out/${w}_dl.jsonl'):
    d=json.loads(l); print('$w', d['plan_name'], d['kernel_ms'], d['groups'])"
  f=$(find $out/${w}_dl_trace -name "*kernel_stats.csv" | head -1); cp $f $out/${w}_dl_kernel_stats.csv
  grep -i walk $out/${w}_dl_kernel_stats.csv || true
done
echo all_ok
