# Round-2 GPU step: chain-kernel parity tests, then config 3 (whole genome) at
# N=1 with a rocprofv3 kernel summary.  Usage: TESTS="..." BENCH=1 PROF=1
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r02}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -5 $OUT/$name.log
  case $rc in 0) return 0;; *) exit $rc;; esac
}
if [ -n "${TESTS:-}" ]; then
  step tests 900 python3 -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread
fi
if [ -n "${BENCH:-}" ]; then
  step bench 900 python3 -u $R/bench.py --workload genome --steps ${STEPS:-10} --warmup 2 ${EXTRA:-}
fi
if [ -n "${PROF:-}" ]; then
  cd /tmp
  step prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 -u $R/bench.py --workload genome --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${EXTRA:-}
  find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
  cat $OUT/kernel_stats.csv | cut -c1-220 | head -12
fi
exit 0
