# Round 6: SQ time-breakdown and instruction-mix counters per kernel for the gdl_jit secondary line (50 %), the
# configs[2] count-free emit + pass C and the configs[4] V / H emits + pass C; kernel trace of configs[4]
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
C2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD"
run() {  # name, command...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc $C1 -d $out/${name}_c1 -o run --output-format csv -- "$@" > $out/${name}_c1.log 2>&1 || { echo ${name}_c1_failed; tail -5 $out/${name}_c1.log; return 1; }
  timeout -s KILL 150 rocprofv3 --pmc $C2 -d $out/${name}_c2 -o run --output-format csv -- "$@" > $out/${name}_c2.log 2>&1 || { echo ${name}_c2_failed; tail -5 $out/${name}_c2.log; return 1; }
  python3 tools/pmc_by_kernel.py $out/${name}_c1 > $out/${name}_c1.json && python3 tools/pmc_by_kernel.py $out/${name}_c2 > $out/${name}_c2.json
}
run gdl50 python3 tools/gdl_sweep.py --segments 30 --settings default --lines sel_50pct --reps 5 || exit 1
run highcard python3 tools/bench_configs.py --workload highcard --plan all_docs --segments 8 --no-stepmajor --reps 3 || exit 2
run star python3 tools/bench_configs.py --workload star --plan all_docs --segments 4 --no-stepmajor --reps 3 || exit 3
PA_DEBUG_PLAN=1 timeout -k 10 200 python3 tools/bench_configs.py --workload star --plan all_docs --segments 4 --no-stepmajor --reps 1 > /dev/null 2> $out/star_plan.err || exit 4
grep -E "pve|partition" $out/star_plan.err | head -10
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/star_trace -o run --output-format csv -- python3 tools/bench_configs.py --workload star --plan all_docs --segments 20 --no-stepmajor --reps 5 > $out/star_trace.json 2> $out/star_trace.err || exit 5
find $out/star_trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $out/star_kernel_stats.csv
head -12 $out/star_kernel_stats.csv | cut -c1-150
for n in gdl50 highcard star; do echo == $n; python3 - <<PY
import json
a=json.load(open('$out/${n}_c1.json')); b=json.load(open('$out/${n}_c2.json'))
for k in a:
    x=dict(a[k]); x.update(b.get(k,{}))
    if x.get('SQ_WAVES',0) < 100 and x.get('SQ_WAVE_CYCLES',0) < 1e6: continue
    keep={c: round(v,3) if isinstance(v,float) else v for c,v in x.items()}
    print(k, json.dumps(keep))
PY
done
echo all_ok
