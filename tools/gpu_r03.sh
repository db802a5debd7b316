# Round-3 validation: smoke, the GPU test suite, the default bench line
# (config 3) and a kernel-trace summary of it.  Each step has its own time
# limit; the first failing step ends the script.
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r03}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.log | cut -c1-400
  case $rc in 0) return 0;; *) exit $rc;; esac
}
if [ -z "$SKIP_TESTS" ]; then
step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()"
step tests 900 python3 -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"}
fi
step bench 600 python3 -u $R/bench.py ${BENCH_ARGS}
if [ -n "$PROF" ]; then
cd /tmp
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS}
fi
exit 0
