# Emit-pass wait isolation (run on the GPU box): kernel ms of one bench_configs plan per PA_DEBUG_EMIT value
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
for d in 0 1 2 4 6 7; do
  PA_DEBUG_EMIT=$d timeout -k 10 300 python3 -u tools/bench_configs.py --no-stepmajor "$@" > $out/dbg$d.json 2> $out/dbg$d.err || { echo "dbg$d failed"; tail -5 $out/dbg$d.err; exit 1; }
  echo "PA_DEBUG_EMIT=$d $(cut -c1-120 $out/dbg$d.json | tr '\n' ' ')"
done
