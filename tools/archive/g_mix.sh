# round-3 combined check: statistics parity + cost + kernel trace, lane / LDS group-by parity + sumgroup timings
set -o pipefail
tag=$1
bash tools/g_stats.sh ${tag}_st && bash tools/g_stats_prof.sh ${tag}_stp && bash tools/g_sg3.sh ${tag}_sg
