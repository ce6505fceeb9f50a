# Round 6: gdl_jit's table lookups at entry 0 for docs no longer matching (PA_GDL_MASK): the dense-path GPU tests, then
# the bench's secondary plans A/B (shared and own dictionaries)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dense.py tests/test_gpu_configs.py -k "dense or gdl or configs1 or secondary or own" > $out/tests.log 2>&1 || { echo tests_failed; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
S=default,nomask,default_b
timeout -k 10 420 python -u tools/gdl_sweep.py --settings $S --reps 10 > $out/mask_shared.jsonl 2> $out/mask_shared.err || { echo shared_failed; tail -5 $out/mask_shared.err; exit 1; }
timeout -k 10 420 python -u tools/gdl_sweep.py --own --settings $S --reps 10 > $out/mask_own.jsonl 2> $out/mask_own.err || { echo own_failed; tail -5 $out/mask_own.err; exit 2; }
python3 -c "import json; [print(d['line'],d['setting'],d['kernel_ms'],d['frac'],d['variant'],d.get('same_groups')) for f in ('$out/mask_shared.jsonl','$out/mask_own.jsonl') for d in map(json.loads,open(f))]"
echo all_ok
