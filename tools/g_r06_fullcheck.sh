# Round 6: the partitioned lines at full size (20 x 10M docs) checked against the oracle (bench_configs.py --check)
set -o pipefail
out=gpurun_out/r06_fullcheck
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {  # workload, extra args
  timeout -k 10 900 python3 -u tools/bench_configs.py --workload $1 --segments 20 --no-stepmajor --warm 5 --reps 10 --check $2 > $out/$1.jsonl 2> $out/$1.err || { echo $1_failed; tail -5 $out/$1.err; exit 1; }
  python3 -c "
import json
for l in open('$out/$1.jsonl'):
    d=json.loads(l); print('$1', d['plan_name'], d['kernel_ms'], d['groups'], d.get('check'))"
}
run ${1:-star} "${2:-}"
echo all_ok
