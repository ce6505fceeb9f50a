# Round 5: launcher line check (stdout = exactly one JSON line) and the headline + one secondary line's counter passes
set -o pipefail
tag=$1; sec=$2
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
if [ "$3" = "launcher" ]; then
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-secondary > $out/launcher.json 2> $out/launcher.err || { echo launcher_failed; tail -20 $out/launcher.err; exit 1; }
python3 -c "
import json; l=open('$out/launcher.json').read().splitlines(); assert len(l)==1, l[:3]; d=json.loads(l[0]); print('launcher', d['value'], d['multi_gpu'])" || exit 2
fi
bash tools/profile.sh ${tag}_$sec --secondary $sec || { echo profile_failed; exit 3; }
date
echo all_ok
