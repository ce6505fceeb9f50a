# sumscan plan decomposition (kernel ms) + SQ/TA counters of sel_10pct and sel_100pct
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/bench_configs.py --workload sumscan --segments 20 --no-stepmajor > $out/ss.json 2> $out/ss.err || { echo fail; tail -5 $out/ss.err; exit 1; }
python3 -c "
import json
for l in open('$out/ss.json'): d=json.loads(l); print(d['plan_name'], d['kernel_ms'], round(d['staged_GBps']))
"
for p in sel_10pct sel_100pct count_100pct; do
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU -d $out/sq_$p -o run --output-format csv -- python3 tools/bench_configs.py --workload sumscan --segments 20 --no-stepmajor --plan $p > /dev/null 2> $out/sq_$p.err || exit 2
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d $out/ta_$p -o run --output-format csv -- python3 tools/bench_configs.py --workload sumscan --segments 20 --no-stepmajor --plan $p > /dev/null 2> $out/ta_$p.err || exit 3
done
echo ok
