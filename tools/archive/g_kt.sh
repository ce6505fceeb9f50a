# Per-plan kernel averages (rocprofv3 kernel trace) of tools/bench_configs.py plans: g_kt.sh tag workload plan...
set -o pipefail
tag=$1; wl=$2; shift 2
out=gpurun_out/kt_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for plan in "$@"; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/$plan -o run --output-format csv -- python3 tools/bench_configs.py --workload $wl --plan $plan --no-stepmajor --reps 3 > $out/$plan.json 2> $out/$plan.err || { echo failed_$plan; exit 1; }
  echo "== $plan"
  python3 -c "
import csv,glob
for f in glob.glob('$out/$plan/**/*kernel_stats.csv', recursive=True):
    for x in list(csv.DictReader(open(f)))[:5]: print('  ', x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e3,1), 'us')"
done
