# Round 5: decomposition of the bench's secondary plan (adanalytics_in, RS8 dense kernel) + LDS op-rate probe.
# PA_DEBUG_EMIT (measurement only, results invalid): 32 = stream only, 1 = filter only, 2 = walk without atomics, 0 = full
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/lds_probe 20000 > $out/lds_probe.txt 2>&1 || { echo probe_failed; cat $out/lds_probe.txt; exit 1; }
cat $out/lds_probe.txt
for plan in sel_10pct sel_50pct; do
  for d in 32 1 2 0; do
    PA_DEBUG_EMIT=$d timeout -k 10 300 python -u tools/bench_configs.py --workload adanalytics_in --plan $plan --segments 30 --no-stepmajor > $out/${plan}_d$d.json 2> $out/${plan}_d$d.err || { echo failed_${plan}_$d; tail -5 $out/${plan}_d$d.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('$out/${plan}_d$d.json').readline()); print('$plan', 'dbg', $d, d['plan_name'], d['kernel_ms'], d['plan']['strategy'], d['plan']['wg_per_cu'], d['plan']['lds_bytes'])"
  done
done
echo all_ok
