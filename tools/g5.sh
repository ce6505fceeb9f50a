# partitioned-aggregation check: its parity tests, then configs[2] (default plan + partition-size sweep)
set -o pipefail
export PYTHONUNBUFFERED=1
tag=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "partition or high_card or highcard or golden or star or mv" > gpurun_out/gpu_tests_$tag.log 2>&1 && \
timeout -k 10 400 python -u tools/bench_configs.py --workload highcard --no-stepmajor --reps 5 > gpurun_out/highcard_$tag.log 2>&1
