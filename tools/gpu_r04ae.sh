# SQ counters of the final request pass (one pass, kernel trace only)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
cd /tmp
timeout -k 10 500 timeout -s KILL 490 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $R/gpurun_out/r04ae/sq -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/r04ae_sq.log 2>&1; rc=$?
echo "rc=$rc"; tail -1 $R/gpurun_out/r04ae_sq.log | cut -c1-200
cd $R && python3 tools/sq_summary.py gpurun_out/r04ae/sq > gpurun_out/r04ae/sq_summary.txt && cat gpurun_out/r04ae/sq_summary.txt | cut -c1-400
exit $rc
