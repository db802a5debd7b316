# SQ counter pass (waves, wait/active cycles, VALU/SALU issue) over the
# config-2 bench and the config-3 genome bench; kernel trace only.
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 $R/gpurun_out/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
cd /tmp
step pmc_sq_c2 300 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $R/gpurun_out/pmc_sq_c2 -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline
step pmc_sq_c3 600 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $R/gpurun_out/pmc_sq_c3 -o run -- python3 $R/bench.py --workload genome --steps 2 --warmup 1 --no-cpu-baseline
exit 0
