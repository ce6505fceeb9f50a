# GPU check: parity tests, planner sweep, headline bench (run on the GPU box from the repo root)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 400 python -u tools/sweep.py --segments 30 --reps 8 > gpurun_out/sweep2.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/bench2.json 2> gpurun_out/bench2.err
