# config-3 bench: delivery digests (step / serial / pipelined) at full size
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04ab}
mkdir -p $OUT
timeout -k 10 600 python3 -u $R/bench.py --no-cpu-baseline > $OUT/genome.log 2>&1; rc=$?
echo "genome rc=$rc"; tail -2 $OUT/genome.log | cut -c1-300
exit $rc
