# Round 6: pass C's H launch with 16 records per thread in flight (PA_PASSC_HKB=16) vs 8, on configs[4]; then the
# configs[2] / configs[4] lines on the current tree (tools/g_r06_cfgfinal.sh)
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for s in hkb16:16 hkb8:8; do
  n=${s%%:*}; v=${s##*:}
  PA_PASSC_HKB=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/star_${n}_trace -o run --output-format csv -- python3 tools/bench_configs.py --workload star --segments 20 --no-stepmajor --reps 10 --plan all_docs > $out/star_${n}.jsonl 2> $out/star_${n}.err || { echo ${n}_failed; tail -5 $out/star_${n}.err; exit 1; }
  python3 -c "
import json
for l in open('$out/star_${n}.jsonl'):
    d=json.loads(l); print('$n', d['plan_name'], d['kernel_ms'], d['groups'])"
  f=$(find $out/star_${n}_trace -name "*kernel_stats.csv" | head -1); cp $f $out/star_${n}_kernel_stats.csv
  grep "part_agg" $out/star_${n}_kernel_stats.csv | cut -c1-150
done
bash tools/g_r06_cfgfinal.sh $tag
