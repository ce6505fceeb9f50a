# Round 6: pass C with two register batches in flight (default) vs one at a time (PA_PASSC_SERIAL=1): partitioned
# parity tests, configs[2] / configs[4] timings + kernel stats; then the gdl_jit knob sweep (tools/g_r06_b5.sh)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_mv.py -x -q --timeout 180 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_failed; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for v in "pipe:" "serial:PA_PASSC_SERIAL=1"; do
  name=${v%%:*}; envs=${v#*:}
  for w in highcard star; do
    env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/${w}_${name}_trace -o run --output-format csv -- python3 tools/bench_configs.py --workload $w --plan all_docs --segments 20 --no-stepmajor --reps 10 > $out/${w}_$name.jsonl 2> $out/${w}_$name.err || { echo ${w}_${name}_failed; tail -5 $out/${w}_$name.err; exit 2; }
    python3 -c "
import json
for l in open('$out/${w}_$name.jsonl'):
    d=json.loads(l); print('$w', '$name', d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'],3), d['plan'].get('count_free_emit'), d['groups'])"
    f=$(find $out/${w}_${name}_trace -name "*kernel_stats.csv" | head -1); cp $f $out/${w}_${name}_kernel_stats.csv
    head -4 $out/${w}_${name}_kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
  done
done
bash tools/g_r06_b5.sh $tag
