# SQ counters of one tools/bench_configs.py plan (run on the GPU box): two passes
set -o pipefail
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAVES -d $out/sq1 -o run --output-format csv -- python3 tools/bench_configs.py "$@" > /dev/null 2> $out/sq1.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_SALU -d $out/sq2 -o run --output-format csv -- python3 tools/bench_configs.py "$@" > /dev/null 2> $out/sq2.err || exit 2
echo sq_ok
