# Round 6: tile-image ring depth (PA_GDL_RING / PA_PVE_RING) on the gdl_jit secondary lines and the count-free emit,
# plus the walk decomposition without row atomics (PA_GDL_DBG=3)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
S=${GDL_SETTINGS:-default,stream_filter,walk_no_atomics,ring3,ring4,ring3_w8_nd16,ring3_w16_nd8,ring3_rr1}
timeout -k 10 420 python -u tools/gdl_sweep.py --settings $S --reps 10 > $out/sweep_shared.jsonl 2> $out/sweep_shared.err || { echo sweep_failed; tail -5 $out/sweep_shared.err; exit 1; }
python3 -c "import sys,json; [print(d['line'],d['setting'],d['kernel_ms'],d['frac'],d['variant'],d['lds_bytes'],d['same_groups']) for d in map(json.loads,open('$out/sweep_shared.jsonl'))]"
timeout -k 10 420 python -u tools/gdl_sweep.py --own --settings $S --reps 10 > $out/sweep_own.jsonl 2> $out/sweep_own.err || { echo sweep_own_failed; tail -5 $out/sweep_own.err; exit 2; }
python3 -c "import sys,json; [print(d['line'],d['setting'],d['kernel_ms'],d['frac'],d['variant'],d['lds_bytes'],d['same_groups']) for d in map(json.loads,open('$out/sweep_own.jsonl'))]"
for r in 2 3 4; do
  PA_PVE_RING=$r timeout -k 10 300 python -u tools/bench_configs.py --workload highcard --plan all_docs --segments 20 --no-stepmajor --reps 10 > $out/highcard_ring$r.jsonl 2> $out/highcard_ring$r.err || { echo highcard_ring${r}_failed; tail -5 $out/highcard_ring$r.err; exit 3; }
  python3 -c "
import json
for l in open('$out/highcard_ring$r.jsonl'):
    d=json.loads(l); print('highcard ring $r', d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'],3), d['plan'].get('count_free_emit'), d['groups'])"
done
echo all_ok
