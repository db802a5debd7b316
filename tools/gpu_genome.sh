# GPU parity tests for the query kernels, then the config-3 (whole-genome,
# contig-sharded) bench at N=1, full size
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -4 $R/gpurun_out/$name.log
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step gpu_tests_q 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_genome.py tests/test_route_golden.py -m gpu -x -v --timeout 300 --timeout-method thread
step genome_full 900 python3 -u $R/bench.py --workload genome --steps ${STEPS:-5} --warmup 1 ${EXTRA:-}
exit 0
