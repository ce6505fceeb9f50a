# Round-3 counters: headline bench (kernel trace, SQ, FETCH_SIZE, WRITE_SIZE passes) + configs[0] 1B-doc lines under
# the kernel trace (frac reproduced from rocprof averages) and their HBM bytes
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/profile.sh $tag > $out/profile.log 2>&1 || { echo profile_failed; tail -5 $out/profile.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_$tag > $out/headline_summary.json || exit 2
for wp in "sumscan sel_10pct" "sumscan sel_50pct" "sumscan_raw sel_10pct" "sumscan_raw sel_50pct"; do
  set -- $wp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kt_$1_$2 -o run --output-format csv -- python3 tools/bench_configs.py --workload $1 --plan $2 --segments 100 --reps 20 --no-stepmajor > $out/kt_$1_$2.json 2> $out/kt_$1_$2.err || { echo kt_failed; exit 3; }
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $out/f_$1_$2 -o run --output-format csv -- python3 tools/bench_configs.py --workload $1 --plan $2 --segments 100 --reps 3 --no-stepmajor > /dev/null 2> $out/f_$1_$2.err || { echo f_failed; exit 4; }
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $out/w_$1_$2 -o run --output-format csv -- python3 tools/bench_configs.py --workload $1 --plan $2 --segments 100 --reps 3 --no-stepmajor > /dev/null 2> $out/w_$1_$2.err || { echo w_failed; exit 5; }
done
echo prof_ok
