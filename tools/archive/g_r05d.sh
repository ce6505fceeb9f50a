# Round 5: lane-major dense walk decomposition on the bench secondary plan (PA_DEBUG_EMIT knobs, results invalid)
set -o pipefail
tag=$1; wl=${2:-adanalytics_in}; plan=${3:-sel_50pct}; segs=${4:-100}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for d in 32 1 2 0; do
  PA_DEBUG_EMIT=$d timeout -k 10 300 python -u tools/bench_configs.py --workload $wl --plan $plan --segments $segs --no-stepmajor > $out/${plan}_d$d.json 2> $out/${plan}_d$d.err || { echo failed_$d; tail -5 $out/${plan}_d$d.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$out/${plan}_d$d.json').readline()); print('$wl $plan', 'dbg', $d, d['kernel_ms'], d['plan']['strategy'], d['plan'].get('variant'), d['plan']['ring'], d['plan']['lds_bytes'])"
done
echo all_ok
