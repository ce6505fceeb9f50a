# numGroupsLimit parity (sorted form: radix select; walk form) + MV group-by limit timings
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "limit or trim or golden" --timeout 300 --timeout-method thread > $out/limit_tests.log 2>&1 || { echo tests_failed; tail -40 $out/limit_tests.log; exit 1; }
tail -3 $out/limit_tests.log
bash tools/g_mvlimit.sh $tag
