# Quick configs[4]/[2] timing on the GPU box (no tests): tools/g_star.sh tag [workload plan]...
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
while [ $# -ge 2 ]; do
  wl=$1; plan=$2; shift 2
  timeout -k 10 200 python -u tools/bench_configs.py --workload $wl --plan $plan --no-stepmajor --reps 5 >> $out/configs.json 2>> $out/configs.err || { echo failed_$wl_$plan; tail -20 $out/configs.err; exit 1; }
done
python3 -c "
import json
for l in open('$out/configs.json'):
    d=json.loads(l); print(d['workload'], d['plan_name'], d['kernel_ms'], d['plan']['wg_per_cu'], d['plan']['lds_bytes'])"
