# Round 6: gdl_jit with 12 waves per workgroup (3 per SIMD) against the default plans on the secondary lines
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
S=${GDL_SETTINGS:-default,w12_nd8,w12_nd16,w8_nd8_pin,w16_nd16}
timeout -k 10 420 python -u tools/gdl_sweep.py --settings $S --reps 10 > $out/sweep_shared.jsonl 2> $out/sweep_shared.err || { echo sweep_failed; tail -5 $out/sweep_shared.err; exit 1; }
python3 -c "import sys,json; [print(d['line'],d['setting'],d['kernel_ms'],d['frac'],d['variant'],d['lds_bytes'],d['dense_packed'],d['same_groups']) for d in map(json.loads,open('$out/sweep_shared.jsonl'))]"
timeout -k 10 420 python -u tools/gdl_sweep.py --own --settings $S --reps 10 > $out/sweep_own.jsonl 2> $out/sweep_own.err || { echo sweep_own_failed; tail -5 $out/sweep_own.err; exit 2; }
python3 -c "import sys,json; [print(d['line'],d['setting'],d['kernel_ms'],d['frac'],d['variant'],d['lds_bytes'],d['dense_packed'],d['same_groups']) for d in map(json.loads,open('$out/sweep_own.jsonl'))]"
echo all_ok
