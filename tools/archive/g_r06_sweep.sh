# Round 6: gdl_jit knob sweep on the bench's shared- and own-dictionary secondary lines, and the partitioned plans'
# shapes (PA_DEBUG_PLAN) of configs[2] / configs[4]
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/gdl_sweep.py "$@" > $out/sweep_shared.jsonl 2> $out/sweep_shared.err || { echo sweep_failed; tail -5 $out/sweep_shared.err; exit 1; }
cat $out/sweep_shared.jsonl | python3 -c "import sys,json; [print(d['line'],d['setting'],d['kernel_ms'],d['frac'],d['variant'],d['dense_packed'],d['same_groups']) for d in map(json.loads,sys.stdin)]"
timeout -k 10 400 python -u tools/gdl_sweep.py --own "$@" > $out/sweep_own.jsonl 2> $out/sweep_own.err || { echo sweep_own_failed; tail -5 $out/sweep_own.err; exit 2; }
cat $out/sweep_own.jsonl | python3 -c "import sys,json; [print(d['line'],d['setting'],d['kernel_ms'],d['frac'],d['variant'],d['dense_packed'],d['same_groups']) for d in map(json.loads,sys.stdin)]"
PA_DEBUG_PLAN=1 timeout -k 10 300 python -u tools/bench_configs.py --workload star --segments 4 --plan all_docs --reps 2 --no-stepmajor > $out/star_plan.jsonl 2> $out/star_plan.err || { echo star_failed; tail -5 $out/star_plan.err; exit 3; }
grep -E "pve|partition|emit" $out/star_plan.err | head -20
echo all_ok
