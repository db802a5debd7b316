# One full GPU pass: smoke, every GPU test, the config-2 bench (+ rocprofv3
# kernel trace), the config-4 paths bench, the config-3 genome bench.
# Stops at the first failing step.
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
STEPS=${STEPS:-20}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 $R/gpurun_out/$name.log | cut -c1-400
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step bench 900 python3 -u $R/bench.py --steps $STEPS --warmup 3
cd /tmp && step prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench -- python3 $R/bench.py --steps $STEPS --warmup 3 --no-cpu-baseline
cd $R && step paths 900 python3 -u $R/bench_paths.py --datasets 10
cd /tmp && step paths_prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/paths_prof -o paths -- python3 $R/bench_paths.py --datasets 10 --steps 5 --no-cpu-baseline
cd $R && step genome 900 python3 -u $R/bench.py --workload genome --steps 5 --warmup 1
exit 0
