# round-3 final tree on the GPU box: g_final.sh (parity, smoke, bench, rocprof, configs lines) + statistics cost +
# filter + GROUP BY SUM timings at 1B docs
set -o pipefail
tag=$1
bash tools/g_final.sh $tag && bash tools/g_stats.sh ${tag}_st && bash tools/g_sg.sh ${tag}_sg
