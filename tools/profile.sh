#!/bin/bash
# rocprofv3 passes for the headline bench (run on the GPU box from the repo root):
#   1) kernel trace + stats   2) SQ stall counters   3) HBM FETCH/WRITE bytes (separate passes, per the guide)
# Usage: bash tools/profile.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
args="$@"
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 bench.py --cpu-sample 0 $args > $out/bench.json 2> $out/bench.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAVES -d $out/sq -o run --output-format csv -- python3 bench.py --cpu-sample 0 $args > /dev/null 2> $out/sq.err || exit 2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run --output-format csv -- python3 bench.py --cpu-sample 0 $args > /dev/null 2> $out/fetch.err || exit 3
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run --output-format csv -- python3 bench.py --cpu-sample 0 $args > /dev/null 2> $out/write.err || exit 4
echo profile_ok
