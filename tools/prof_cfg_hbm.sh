# kernel trace + HBM write bytes of the configs[2] partitioned plan (run on the GPU box)
set -o pipefail
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 tools/bench_configs.py "$@" > $out/out.json 2> $out/err.log || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run --output-format csv -- python3 tools/bench_configs.py "$@" > /dev/null 2> $out/write.err || exit 2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run --output-format csv -- python3 tools/bench_configs.py "$@" > /dev/null 2> $out/fetch.err || exit 3
echo prof_ok
