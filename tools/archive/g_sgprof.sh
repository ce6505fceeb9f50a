# SQ counters of the filter + GROUP BY SUM (LDS strategy) kernel at 50 % selectivity, 200M docs
set -o pipefail
tag=$1; wl=${2:-sumgroup}; pl=${3:-sel_50pct}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU -d $out/sq -o run --output-format csv -- python3 tools/bench_configs.py --workload $wl --plan $pl --segments 20 --reps 3 --no-stepmajor > /dev/null 2> $out/sq.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVES -d $out/sq2 -o run --output-format csv -- python3 tools/bench_configs.py --workload $wl --plan $pl --segments 20 --reps 3 --no-stepmajor > /dev/null 2> $out/sq2.err || exit 2
python3 tools/pmc_by_kernel.py $out/sq | grep -A14 "scan_kernel"
python3 tools/pmc_by_kernel.py $out/sq2 | grep -A10 "scan_kernel"
