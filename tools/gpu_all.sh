# smoke -> gpu tests -> bench -> rocprofv3 kernel trace; stops at the first
# fault/abort/timeout (exit codes other than 0/1)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
STEPS=${STEPS:-20}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -4 $R/gpurun_out/$name.log
  case $rc in 0|1) return 0;; *) exit $rc;; esac
}
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step bench 900 python3 $R/bench.py --steps $STEPS --warmup 3
cp $R/gpurun_out/bench.log $R/gpurun_out/bench_full.log
cd /tmp && step prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench -- python3 $R/bench.py --steps $STEPS --warmup 3 --no-cpu-baseline
exit 0
