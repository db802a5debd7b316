mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 $R/gpurun_out/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step gpu_tests 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_genome.py tests/test_route_golden.py -m gpu -x -v --timeout 300 --timeout-method thread
step bench 600 python3 -u $R/bench.py --steps 20 --warmup 3
step genome 900 python3 -u $R/bench.py --workload genome --steps 5 --warmup 1 --no-cpu-baseline
