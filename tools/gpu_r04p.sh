# delivered path sweep + cold-launch probe (tools/delivered_sweep.py)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04p}
mkdir -p $OUT
timeout -k 10 600 python3 -u $R/tools/delivered_sweep.py > $OUT/sweep.log 2>&1; rc=$?
grep "^{" $OUT/sweep.log
exit $rc
