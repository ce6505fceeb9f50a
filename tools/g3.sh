# GPU check: parity tests, headline bench, rocprof passes (run on the GPU box from the repo root)
set -o pipefail
export PYTHONUNBUFFERED=1
tag=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err && \
bash tools/profile.sh $tag --steps 10 --warmup 2 && \
python tools/prof_summary.py gpurun_out/prof_$tag > gpurun_out/prof_${tag}_summary.json
