# Round 5: statistics engine tests + a timing of the statistics call on the bench's secondary plan (1B docs)
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_stats.py tests/test_gpu_parity.py -k "stats or golden" -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_failed; grep -E "FAILED|Error|assert" $out/tests.log | head -30; tail -5 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python -u tools/bench_configs.py --workload adanalytics_in --segments 100 --no-stepmajor --reps 5 --exec-stats > $out/exec_stats.json 2> $out/exec_stats.err || { echo bench_failed; tail -20 $out/exec_stats.err; exit 2; }
python3 -c "
import json
for l in open('$out/exec_stats.json'):
    d=json.loads(l); print(d['plan_name'], d['kernel_ms'], d['exec_stats'])"
echo all_ok
