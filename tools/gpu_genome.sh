# GPU tests, then the config-3 (whole-genome, contig-sharded) bench at N=1:
# a reduced size first, then the full 85 M records / 1 M requests.
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -4 $R/gpurun_out/$name.log
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step gpu_tests 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step genome_small 600 python3 -u $R/bench.py --workload genome --genome-records 10000000 --genome-requests 100000 --steps 5 --warmup 1 --cpu-seconds 5
step genome_full 900 python3 -u $R/bench.py --workload genome --steps 5 --warmup 1
exit 0
