# GPU parity tests + bench under torch.distributed.run (world 1: RCCL merge path) + plain bench
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo tests_failed; tail -40 $out/gpu_tests.log; exit 1; }
tail -2 $out/gpu_tests.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --cpu-sample 0 > $out/bench_dist.json 2> $out/bench_dist.err || { echo dist_bench_failed; tail -30 $out/bench_dist.err; exit 2; }
cat $out/bench_dist.json | cut -c1-300
timeout -k 10 300 python -u bench.py > $out/bench.json 2> $out/bench.err || { echo bench_failed; tail -20 $out/bench.err; exit 3; }
cat $out/bench.json
echo all_ok
