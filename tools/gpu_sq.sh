# SQ instruction / wait counters for the scan kernel, default vs no-multiallelic store
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES"
timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/sq_default -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/sq_default.log 2>&1 || exit $?
SBS_MULTI_FRAC=0 timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/sq_nomulti -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/sq_nomulti.log 2>&1 || exit $?
