# bench + rocprofv3 kernel-trace summary (round-1 measurement)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
STEPS=${STEPS:-20}
timeout -k 10 900 python3 $R/bench.py --steps $STEPS --warmup 3 > $R/gpurun_out/bench.json 2> $R/gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; cat $R/gpurun_out/bench.json; tail -5 $R/gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench -- python3 $R/bench.py --steps $STEPS --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err; rc=$?
echo "prof rc=$rc"; ls -R $R/gpurun_out/prof | head -20
exit $rc
