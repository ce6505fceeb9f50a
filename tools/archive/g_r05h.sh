# Round 5: SQ counters, prototype (tools/mc_probe) vs product lane-major walk, bench secondary shape
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for m in 2 3; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAVES -d $out/p$m/sq1 -o run --output-format csv -- ./tools/mc_probe 200000000 $m > $out/p$m.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_SALU -d $out/p$m/sq2 -o run --output-format csv -- ./tools/mc_probe 200000000 $m >> $out/p$m.log 2>&1 || exit 2
  python3 tools/pmc_by_kernel.py $out/p$m > $out/p$m/summary.json
  python3 -c "
import json; d=json.load(open('$out/p$m/summary.json'))
for k,v in d.items(): print('proto mode $m', k[:30], {c: v.get(c) for c in ('dispatches','SQ_WAVES','SQ_INSTS_VALU','SQ_INSTS_SALU','SQ_INSTS_LDS','SQ_LDS_BANK_CONFLICT','frac_WAIT_ANY','frac_ACTIVE_INST_ANY','frac_ACTIVE_INST_VALU','SQ_WAVE_CYCLES')})
"
done
for d in 1 0; do
  PA_DEBUG_EMIT=$d bash tools/prof_cfg_sq.sh ${tag}_d$d --workload adanalytics_in --plan sel_50pct --segments 20 --no-stepmajor --reps 3 || { echo prof_failed_$d; exit 1; }
  python3 tools/pmc_by_kernel.py gpurun_out/prof_${tag}_d$d > gpurun_out/prof_${tag}_d$d/summary.json
  python3 -c "
import json; d=json.load(open('gpurun_out/prof_${tag}_d$d/summary.json'))
for k,v in d.items():
    if 'gdense' in k: print('product dbg $d', k[:30], {c: v.get(c) for c in ('dispatches','SQ_WAVES','SQ_INSTS_VALU','SQ_INSTS_SALU','SQ_INSTS_LDS','SQ_LDS_BANK_CONFLICT','frac_WAIT_ANY','frac_ACTIVE_INST_ANY','frac_ACTIVE_INST_VALU','SQ_WAVE_CYCLES')})
"
done
echo all_ok
