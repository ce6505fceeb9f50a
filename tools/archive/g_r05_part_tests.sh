# Round 5: every partitioned / numGroupsLimit / MV / configs parity test
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_mv.py -k "partition or limit or configs or mv or group" -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_failed; grep -E "FAILED|Error|assert" $out/tests.log | head -30; tail -5 $out/tests.log; exit 1; }
tail -2 $out/tests.log
echo all_ok
