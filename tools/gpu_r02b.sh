# Round-2 re-validation after a container restore: smoke, every GPU test,
# config 3 bench + rocprofv3 kernel summary, config 4 paths bench (50 ds).
# Stops at the first failing step.
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r02b}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.log | cut -c1-600
  case $rc in 0) return 0;; *) exit $rc;; esac
}
[ -n "${NO_SMOKE:-}" ] || step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()"
[ -n "${NO_TESTS:-}" ] || step gpu_tests 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
[ -n "${NO_BENCH:-}" ] || step bench 900 python3 -u $R/bench.py --steps ${STEPS:-20} --warmup 3
if [ -n "${PROF:-}" ]; then
  cd /tmp && step prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 $R/bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline
  find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
  cd $R
fi
[ -z "${PATHS:-}" ] || step paths 900 python3 -u $R/bench_paths.py --datasets 50
exit 0
