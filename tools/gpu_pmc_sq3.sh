# SQ counter pass over the config-3 genome bench (kernel trace only)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
cd /tmp
timeout -k 10 600 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $R/gpurun_out/pmc_sq_c3 -o run -- python3 $R/bench.py --workload genome --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_sq_c3.log 2>&1; rc=$?
echo "rc=$rc"; tail -2 $R/gpurun_out/pmc_sq_c3.log | cut -c1-200
exit $rc
