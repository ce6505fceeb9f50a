# GPU parity tests without -x: every failure listed (run on the GPU box from the repo root)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread "$@" > $out/gpu_tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $out/gpu_tests.log | cut -c1-300 | tail -60
exit $rc
