# one call: request/wire tests, config-3 bench + kernel trace, wire split, SQ counters
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r03l}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.log | cut -c1-400
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 400 python3 -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread -k "requests or genome or wire or chains"
step bench 600 python3 -u $R/bench.py --no-cpu-baseline
SBEACON_WIRE_TRACE=1 step wire 300 python3 -u $R/tools/wire_split.py
cd /tmp
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
SQ2="SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU"
step sq1 400 timeout -s KILL 390 rocprofv3 --pmc $SQ1 --kernel-trace --output-format csv -d $OUT/sq1 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
step sq2 400 timeout -s KILL 390 rocprofv3 --pmc $SQ2 --kernel-trace --output-format csv -d $OUT/sq2 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
exit 0
