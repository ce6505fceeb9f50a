# GPU check after a kernel change: parity tests, quick plan sweep, headline bench
set -o pipefail
export PYTHONUNBUFFERED=1
tag=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1 && \
timeout -k 10 300 python -u tools/sweep.py --segments 100 --reps 10 --quick > gpurun_out/sweep_$tag.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
