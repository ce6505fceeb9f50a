# Round 6: counter passes (kernel trace, SQ, FETCH_SIZE, WRITE_SIZE) of the given secondary lines, one bench run each
set -o pipefail
tag=$1; shift
for sec in "$@"; do
  bash tools/profile.sh ${tag}_$sec --secondary $sec || { echo profile_failed_$sec; exit 3; }
  python3 tools/pmc_write.py gpurun_out/prof_${tag}_$sec adanalytics_in_list_$sec gdl_jit 10000000 100 jit gpurun_out/prof_${tag}_$sec/pmc.json || exit 4
done
echo all_ok
