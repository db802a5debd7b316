# window_dedupe_kernel ablations (tools/dedup_ablate.py)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04i}
mkdir -p $OUT
timeout -k 10 500 python3 -u $R/tools/dedup_ablate.py > $OUT/ablate.log 2>&1; rc=$?
cat $OUT/ablate.log | grep mode
exit $rc
