# kernel-trace profile of one tools/bench_configs.py plan (run on the GPU box)
set -o pipefail
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 tools/bench_configs.py "$@" > $out/out.json 2> $out/err.log
