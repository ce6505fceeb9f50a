# Round 5: configs[2] / configs[4] partitioned plan sweep (emit workgroup size, resident-wave target, pass-C LDS)
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {  # name, env..., -- args
  name=$1; shift
  env "$@" timeout -k 10 240 python -u tools/bench_configs.py --segments 20 --no-stepmajor --reps 10 $ARGS > $out/$name.json 2> $out/$name.err || { echo "$name failed"; tail -5 $out/$name.err; return 1; }
  python3 -c "
import json
for l in open('$out/$name.json'):
    d=json.loads(l); print('$name', d['workload'], d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'],3), d['plan'].get('grid'), d['plan'].get('wg_per_cu'), d['plan'].get('lds_bytes'))"
}
ARGS="--workload highcard --plan all_docs"
run hc_base PA_X=0 || exit 1
run hc_big1 PA_EMIT_BIG=1 || exit 1
run hc_big0 PA_EMIT_BIG=0 || exit 1
run hc_w16 PA_EMIT_MIN_WAVES=16 || exit 1
run hc_w16b PA_EMIT_MIN_WAVES=16 PA_EMIT_BIG=1 || exit 1
run hc_w32b PA_EMIT_MIN_WAVES=32 PA_EMIT_BIG=1 || exit 1
ARGS="--workload highcard --plan all_docs --sweep-part"
run hc_sweep PA_X=0 || exit 1
ARGS="--workload star --plan all_docs"
run st_base PA_X=0 || exit 1
run st_big1 PA_EMIT_BIG=1 || exit 1
run st_w16b PA_EMIT_MIN_WAVES=16 PA_EMIT_BIG=1 || exit 1
echo all_ok
