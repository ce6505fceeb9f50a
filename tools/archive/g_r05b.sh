# Round 5: lane-major dense GROUP BY prototype (tools/mc_probe.hip) on the bench secondary shape
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 240 ./tools/mc_probe 1000000000 > $out/mc_probe.txt 2>&1 || { echo probe_failed; cat $out/mc_probe.txt; exit 1; }
cat $out/mc_probe.txt
