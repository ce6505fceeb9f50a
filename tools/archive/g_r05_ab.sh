# Round 5: headline A/B on one box (default flags vs the given flags), kernel stats of both
set -o pipefail
tag=$1; flags=$2
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for f in 0 $flags 0 $flags; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-sample 0 --no-secondary --flags $f > $out/bench_$f.json 2> $out/bench_$f.err || { echo bench_failed; tail -20 $out/bench_$f.err; exit 2; }
python3 -c "
import json; d=json.loads(open('$out/bench_$f.json').readline())
print('flags $f', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],3), d['stats_step']['ms_per_step'], d['stats_step']['fused'])"
done
echo all_ok
