# Round-4 correctness batch: fused statistics, multi-rank merges, two-word keys + the hashed / parity suite, dense kernel
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_stats.py tests/test_gpu_dist.py tests/test_gpu_dense.py "tests/test_gpu_parity.py::test_group_keys_wider_than_64_bits" "tests/test_gpu_parity.py::test_raw_group_by_hashed" "tests/test_gpu_parity.py::test_hashed_dictionary_key_space" -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_failed; grep -E "PASSED|FAILED|Error|error" $out/tests.log | tail -30; tail -60 $out/tests.log; exit 1; }
grep -c PASSED $out/tests.log
tail -2 $out/tests.log
echo all_ok
