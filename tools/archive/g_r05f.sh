# Round 5: lane-major dense walk: compute-only decomposition (PA_DEBUG_EMIT 64 = no DMA) of the bench secondary plan
set -o pipefail
tag=$1; plan=${2:-sel_50pct}; flags=${3:-0}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for d in 32 1 2 0 65 66 64; do
  PA_DEBUG_EMIT=$d timeout -k 10 300 python -u tools/bench_configs.py --workload adanalytics_in --plan $plan --segments 100 --no-stepmajor --flags $flags > $out/${plan}_d$d.json 2> $out/${plan}_d$d.err || { echo failed_$d; tail -5 $out/${plan}_d$d.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$out/${plan}_d$d.json').readline()); print('adanalytics_in $plan', 'dbg', $d, d['kernel_ms'], d['plan'].get('variant'), d['plan'].get('dense_packed'))"
done
echo all_ok
