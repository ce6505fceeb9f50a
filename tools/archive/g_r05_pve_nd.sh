# Round 5: count-free emit, 8 vs 16 docs per lane: parity and configs[2] timings
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for nd in 8 16; do
  PA_PVE_ND=$nd timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -k "configs2" -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests_$nd.log 2>&1 || { echo "tests $nd failed"; grep -E "FAILED|Error|assert" gpurun_out/${tag}_tests_$nd.log | head -20; exit 1; }
  tail -1 gpurun_out/${tag}_tests_$nd.log
done
VARIANTS="nd8:PA_PVE_ND=8 nd16:PA_PVE_ND=16" bash tools/g_r05_pve_dec.sh $tag || exit 2
echo all_ok
