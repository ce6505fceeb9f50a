# Emit-pass occupancy sweep (PA_EMIT_MIN_WAVES: resident waves per CU the planner wants before keeping larger bins)
set -o pipefail
out=gpurun_out/emit_sweep
mkdir -p $out
for w in 8 12 16 24 32; do
  for wl in highcard star; do
    PA_EMIT_MIN_WAVES=$w timeout -k 10 200 python -u tools/bench_configs.py --workload $wl --plan all_docs --no-stepmajor --reps 3 > $out/${wl}_$w.json 2> $out/${wl}_$w.err || { echo failed_$wl_$w; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/${wl}_$w.json').readline()); print('$w', d['workload'], d['kernel_ms'], d['plan']['wg_per_cu'], d['plan']['lds_bytes'])"
  done
done
