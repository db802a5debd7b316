# config 5: GPU parity test for attached carrier planes, then the gnomAD-shape
# bench at reduced and full size (shard 0 of 8 on one GPU)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -6 $R/gpurun_out/$name.log
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step gnomad_test 300 python3 -u -m pytest tests/test_gnomad.py -m gpu -x -v --timeout 240 --timeout-method thread
step gnomad_small 400 python3 -u $R/bench.py --workload gnomad --gnomad-records 75000000 --steps 10 --warmup 2 --cpu-seconds 6
[ "${FULL:-1}" = 1 ] && step gnomad_full 900 python3 -u $R/bench.py --workload gnomad --steps 10 --warmup 2
exit 0
