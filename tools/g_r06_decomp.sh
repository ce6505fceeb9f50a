# Round 6: gdl_jit decomposition on the bench's own secondary plans (shared and own dictionaries): stream only /
# + filter / + group keys and packed terms without the row atomics / full (PA_GDL_DBG 1 / 2 / 3; results invalid)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
S=default,stream_only,stream_filter,walk_no_atomics
timeout -k 10 420 python -u tools/gdl_sweep.py --settings $S --reps 10 > $out/decomp_shared.jsonl 2> $out/decomp_shared.err || { echo shared_failed; tail -5 $out/decomp_shared.err; exit 1; }
timeout -k 10 420 python -u tools/gdl_sweep.py --own --settings $S --reps 10 > $out/decomp_own.jsonl 2> $out/decomp_own.err || { echo own_failed; tail -5 $out/decomp_own.err; exit 2; }
python3 -c "import json; [print(d['line'],d['setting'],d['kernel_ms'],d['frac'],d['variant']) for f in ('$out/decomp_shared.jsonl','$out/decomp_own.jsonl') for d in map(json.loads,open(f))]"
echo all_ok
