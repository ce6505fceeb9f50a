# configs[2] / configs[4] lines + per-kernel times under rocprofv3 (run on the GPU box from the repo root)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/bench_configs.py --no-stepmajor "$@" > $out/configs.json 2> $out/configs.err || { echo configs_failed; tail -20 $out/configs.err; exit 1; }
cut -c1-300 $out/configs.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 tools/bench_configs.py --no-stepmajor "$@" > /dev/null 2> $out/prof.err || { echo prof_failed; exit 2; }
python3 -c "import csv,glob; r=[x for f in glob.glob(\"$out/trace/**/*kernel_stats.csv\", recursive=True) for x in csv.DictReader(open(f))]; [print(x[\"Name\"][:70], x[\"Calls\"], round(float(x[\"AverageNs\"])/1e3,1), \"us\") for x in r[:14]]"
echo configs_ok
