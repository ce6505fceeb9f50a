# Dense GROUP BY cost decomposition (measurement only, results invalid): PA_DEBUG_EMIT knobs of pa_gdense.h
# 1 = filter only, 2 = no LDS atomics, 4 = no value-table reads, 8 = always the sparse walk, 16 = always the dense walk
set -o pipefail
tag=$1; wl=${2:-sumgroup_dict}; plan=${3:-sel_50pct}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for d in ${KNOBS:-0 1 2 4 6}; do
  PA_DEBUG_EMIT=$d timeout -k 10 200 python -u tools/bench_configs.py --workload $wl --plan $plan --segments ${SEGS:-30} --no-stepmajor > $out/d$d.json 2> $out/d$d.err || { echo failed_$d; tail -5 $out/d$d.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$out/d$d.json').readline()); print('dbg', $d, d['plan_name'], d['kernel_ms'], d['matched_docs'])"
done
echo all_ok
