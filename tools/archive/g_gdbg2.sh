# Dense GROUP BY streaming decomposition (measurement only, results invalid): PA_DEBUG_EMIT 32 = stream the tiles only,
# 1 = filter only, 0 = full; register-staged (default plan) and LDS-DMA ring (PA_QF_NO_REG_STAGE) variants
set -o pipefail
tag=$1; wl=${2:-sumgroup_dict}; plan=${3:-sel_50pct}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for fl in 0 262144; do
  for d in 32 1 0; do
    PA_DEBUG_EMIT=$d timeout -k 10 200 python -u tools/bench_configs.py --workload $wl --plan $plan --segments 30 --no-stepmajor --flags $fl > $out/f${fl}_d$d.json 2> $out/f${fl}_d$d.err || { echo failed_$fl_$d; tail -5 $out/f${fl}_d$d.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('$out/f${fl}_d$d.json').readline()); print('flags', $fl, 'dbg', $d, d['plan_name'], d['kernel_ms'], d['plan']['strategy'], d['plan']['ring'], d['plan']['wg_per_cu'])"
  done
done
echo all_ok
