# Kernel trace + SQ and HBM counters, per kernel, of one tools/bench_configs.py selection (run on the GPU box)
set -o pipefail
tag=$1; shift
out=gpurun_out/pmc_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" -d $out/$n -o run --output-format csv -- python3 tools/bench_configs.py --no-stepmajor $ARGS > /dev/null 2> $out/$n.err
}
ARGS="$*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 tools/bench_configs.py --no-stepmajor $ARGS > $out/out.json 2> $out/trace.err || { echo trace_failed; exit 1; }
python3 -c "import csv,glob; r=[x for f in glob.glob(\"$out/trace/**/*kernel_stats.csv\", recursive=True) for x in csv.DictReader(open(f))]; [print(x[\"Name\"][:80], x[\"Calls\"], round(float(x[\"AverageNs\"])/1e3,1), \"us\") for x in r[:14]]"
run sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAVES || { echo sq1_failed; exit 2; }
run sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU || { echo sq2_failed; exit 3; }
run fetch FETCH_SIZE || { echo fetch_failed; exit 4; }
run write WRITE_SIZE || { echo write_failed; exit 5; }
python3 tools/pmc_by_kernel.py $out > $out/pmc.json && echo pmc_ok
