# GPU tests, config-5 bench at full size, rocprofv3 kernel summary of the same
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -4 $R/gpurun_out/$name.log
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step gpu_tests 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread
step gnomad_full 600 python3 -u $R/bench.py --workload gnomad --steps 20 --warmup 3
cd /tmp && step gnomad_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/gprof -o gnomad -- python3 $R/bench.py --workload gnomad --steps 20 --warmup 3 --no-cpu-baseline
exit 0
