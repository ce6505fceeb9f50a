# Round 6: gdl_jit plan knobs on bench.py's secondary lines, timed after 20 warm scans (clocks at steady state)
set -o pipefail
out=gpurun_out/r06_warmsweep
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
S=default,w12_nd8,w16_nd8_rs2,w8_nd16_rs2,w16_nd8,ring3,rr1,w12_nd16,default_b
timeout -k 10 400 python -u tools/gdl_sweep.py --warm 20 --reps 50 --settings $S > $out/shared.jsonl 2> $out/shared.err || { echo shared_failed; tail -20 $out/shared.err; exit 1; }
timeout -k 10 400 python -u tools/gdl_sweep.py --own --warm 20 --reps 50 --settings $S > $out/own.jsonl 2> $out/own.err || { echo own_failed; tail -20 $out/own.err; exit 2; }
python3 -c "
import json
for f in ('shared','own'):
    for l in open('$out/%s.jsonl' % f):
        d=json.loads(l); print(f, d['line'], d['setting'], d['kernel_ms'], d['frac'], d['lds_bytes'], d['same_groups'])
"
