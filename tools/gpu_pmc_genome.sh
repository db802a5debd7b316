# PMC passes (one counter group per run) over the config-3 genome bench
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
ARGS="--workload genome --steps 2 --warmup 1 --no-cpu-baseline ${EXTRA:-}"
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 $R/gpurun_out/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
cd /tmp
step pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU --kernel-trace --output-format csv -d $R/gpurun_out/pmc_g_sq -o run -- python3 $R/bench.py $ARGS
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_g_fetch -o run -- python3 $R/bench.py $ARGS
step pmc_tcc 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $R/gpurun_out/pmc_g_tcc -o run -- python3 $R/bench.py $ARGS
exit 0
