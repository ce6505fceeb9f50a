# Round-4 final, part B: configs lines on one byte model (configs[0]-shape GROUP BY at 1B docs, configs[1]-shape
# secondary lines, configs[2], configs[4], MV GROUP BY), the fused statistics, per-kernel averages
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for spec in "sumgroup 100" "sumgroup_dict 100" "adanalytics_in 100" "highcard 20" "star 20" "mvgroup 20"; do
  set -- $spec
  timeout -k 10 400 python -u tools/bench_configs.py --workload $1 --segments $2 --no-stepmajor > $out/configs_$1.json 2> $out/configs_$1.err || { echo configs_failed $1; tail -20 $out/configs_$1.err; exit 1; }
  python3 -c "import json; [print(d['workload'], d['plan_name'], d['kernel_ms'], round(d['roofline']['frac'], 3), d['plan']['strategy']) for d in map(json.loads, open('$out/configs_$1.json'))]"
done
timeout -k 10 400 python -u tools/bench_configs.py --workload adanalytics --segments 100 --no-stepmajor --exec-stats > $out/exec_stats_adanalytics.json 2> $out/exec_stats.err || { echo stats_failed; tail -20 $out/exec_stats.err; exit 2; }
timeout -k 10 400 python -u tools/bench_configs.py --workload sumscan --plan sel_10pct --segments 100 --no-stepmajor --exec-stats > $out/exec_stats_sumscan.json 2>> $out/exec_stats.err || { echo stats_failed; exit 2; }
cat $out/exec_stats_*.json | python3 -c "import json,sys; [print(d['workload'], d['plan_name'], d['exec_stats']) for d in map(json.loads, sys.stdin)]"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/stats_trace -o run --output-format csv -- python3 tools/bench_configs.py --workload adanalytics --segments 100 --reps 10 --no-stepmajor --exec-stats > /dev/null 2> $out/stats_trace.err || { echo stats_prof_failed; exit 3; }
for w in highcard star mvgroup; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/kt_$w -o run --output-format csv -- python3 tools/bench_configs.py --workload $w --plan $([ $w = mvgroup ] && echo untrimmed || echo all_docs) --segments 20 --no-stepmajor > /dev/null 2> $out/kt_$w.err || { echo kt_failed $w; exit 4; }
done
echo all_ok
