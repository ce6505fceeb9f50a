# SQ time-breakdown counters for one sweep configuration, full vs stream-only (run on the GPU box)
set -o pipefail
tag=$1; cfg=${2:-auto}
out=gpurun_out/pmc_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
for mode in full stream; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $out/$mode -o run --output-format csv -- python3 tools/sweep.py --segments 100 --reps 10 --only $cfg --mode $mode > $out/$mode.log 2> $out/$mode.err || exit 1
done
echo pmc_ok
