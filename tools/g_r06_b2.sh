# Round 6: gdl_jit hoisted column reads (PA_GDL_HOIST) and row sharing; the count-free emit's double-buffered bins
# (PA_PVE_DB): parity tests first, then configs[2] / configs[4] timings
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PA_PVE_DB=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -k "configs2 or configs4" -x -v --timeout 180 --timeout-method thread > $out/db_tests.log 2>&1 || { echo db_tests_failed; tail -30 $out/db_tests.log; exit 1; }
tail -3 $out/db_tests.log
for v in "base:" "db:PA_PVE_DB=1"; do
  name=${v%%:*}; envs=${v#*:}
  for w in highcard star; do
    env $envs timeout -k 10 300 python -u tools/bench_configs.py --workload $w --plan all_docs --segments 20 --no-stepmajor --reps 10 > $out/${w}_$name.jsonl 2> $out/${w}_$name.err || { echo ${w}_${name}_failed; tail -5 $out/${w}_$name.err; exit 2; }
    python3 -c "
import json
for l in open('$out/${w}_$name.jsonl'):
    d=json.loads(l); print('$w', '$name', d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'],3), d['plan'].get('count_free_emit'), d['groups'])"
  done
done
S=${GDL_SETTINGS:-default,no_hoist,walk_no_atomics,w16_nd8_rs2,w8_nd16_rs2}
timeout -k 10 420 python -u tools/gdl_sweep.py --settings $S --reps 10 > $out/sweep_shared.jsonl 2> $out/sweep_shared.err || { echo sweep_failed; tail -5 $out/sweep_shared.err; exit 3; }
python3 -c "import sys,json; [print(d['line'],d['setting'],d['kernel_ms'],d['frac'],d['variant'],d['lds_bytes'],d['same_groups']) for d in map(json.loads,open('$out/sweep_shared.jsonl'))]"
timeout -k 10 420 python -u tools/gdl_sweep.py --own --settings $S --reps 10 > $out/sweep_own.jsonl 2> $out/sweep_own.err || { echo sweep_own_failed; tail -5 $out/sweep_own.err; exit 4; }
python3 -c "import sys,json; [print(d['line'],d['setting'],d['kernel_ms'],d['frac'],d['variant'],d['lds_bytes'],d['same_groups']) for d in map(json.loads,open('$out/sweep_own.jsonl'))]"
echo all_ok
