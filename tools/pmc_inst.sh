# instruction-mix counters: real scan kernel (auto plan, full) vs the HBM probe's lane-major mimic (run on the GPU box)
set -o pipefail
out=gpurun_out/pmc_inst
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD"
timeout -s KILL 120 rocprofv3 --pmc $C -d $out/real -o run --output-format csv -- python3 tools/sweep.py --segments 100 --reps 5 --only auto --mode full > $out/real.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $C -d $out/probe -o run --output-format csv -- ./tools/hbm_probe 2125081600 random > $out/probe.log 2>&1 || exit 2
echo ok
