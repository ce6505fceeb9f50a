# Emit-pass cost decomposition (measurement only, results invalid): PA_DEBUG_EMIT bit 0 skips record stores, bit 1 the
# HLL LUT gathers, bit 2 the MV value reads. g_emit_dbg.sh tag workload plan
set -o pipefail
tag=$1; wl=$2; plan=$3
out=gpurun_out/emitdbg_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for d in 0 1 2 4 6 7; do
  PA_DEBUG_EMIT=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/d$d -o run --output-format csv -- python3 tools/bench_configs.py --workload $wl --plan $plan --no-stepmajor --reps 3 > $out/d$d.json 2> $out/d$d.err || { echo failed_$d; exit 1; }
  echo "== PA_DEBUG_EMIT=$d"
  python3 -c "
import csv,glob
for f in glob.glob('$out/d$d/**/*kernel_stats.csv', recursive=True):
    for x in list(csv.DictReader(open(f)))[:4]: print('  ', x['Name'][:50], round(float(x['AverageNs'])/1e3,1), 'us')"
done
