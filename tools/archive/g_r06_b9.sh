# Round 6: compacted put rounds (PA_PVE_Q=1: per-wave record queue in LDS) in the count-free emit: partitioned parity
# tests with the queue on, then configs[2] (every plan) / configs[4] timings with it off / on, per-kernel durations
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PA_PVE_Q=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_mv.py -x -q --timeout 180 --timeout-method thread > $out/tests_q.log 2>&1 || { echo tests_q_failed; tail -30 $out/tests_q.log; exit 1; }
tail -2 $out/tests_q.log
for v in "base:" "q:PA_PVE_Q=1"; do
  name=${v%%:*}; envs=${v#*:}
  for w in star highcard; do
    plan="--plan all_docs"; [ $w = highcard ] && plan=""
    env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/${w}_${name}_trace -o run --output-format csv -- python3 tools/bench_configs.py --workload $w $plan --segments 20 --no-stepmajor --reps 10 > $out/${w}_$name.jsonl 2> $out/${w}_$name.err || { echo ${w}_${name}_failed; tail -5 $out/${w}_$name.err; exit 2; }
    python3 -c "
import json
for l in open('$out/${w}_$name.jsonl'):
    d=json.loads(l); print('$w', '$name', d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'],3), d['plan'].get('count_free_emit'), d['groups'])"
    f=$(find $out/${w}_${name}_trace -name "*kernel_trace.csv" | head -1)
    python3 - "$f" <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "pve_jit" in n or "part_agg" in n:
        d[n[:40]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in d.items():
    v = sorted(v)
    print("   ", n, "n", len(v), "us min %.0f median %.0f max %.0f" % (v[0], v[len(v) // 2], v[-1]))
PY
  done
done
echo all_ok
