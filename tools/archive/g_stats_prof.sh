# kernel trace of the execution statistics at configs[1] scale (per-kernel durations of the batched count pass)
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 tools/bench_configs.py --workload adanalytics --segments 100 --reps 10 --no-stepmajor --exec-stats > $out/stats.json 2> $out/stats.err || { echo bench_failed; tail -5 $out/stats.err; exit 1; }
cat $out/stats.json
f=$(find $out/prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-5 "$f" | head -20
