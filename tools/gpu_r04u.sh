# delivered-path diagnostics: device planner phase trace + pipelined chunk timeline
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04u}
mkdir -p $OUT
timeout -k 10 500 python3 -u $R/tools/delivered_timeline.py > $OUT/timeline.log 2>&1; rc=$?
echo "timeline rc=$rc"; tail -3 $OUT/timeline.log | cut -c1-300
exit $rc
