# config-2 bench line (wire figure as the steady-state median)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04z}
mkdir -p $OUT
timeout -k 10 500 python3 -u $R/bench.py --workload chr22 --cpu-seconds 8 > $OUT/chr22.log 2>&1; rc=$?
echo "chr22 rc=$rc"; tail -1 $OUT/chr22.log | cut -c1-300
exit $rc
