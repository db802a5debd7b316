# request/wire tests, config-3 bench + kernel trace, config-2 bench (wire line)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r03d}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.log | cut -c1-600
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 400 python3 -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread -k "requests or genome or chains or shard or wire"
step genome 600 python3 -u $R/bench.py --no-cpu-baseline
step chr22 600 python3 -u $R/bench.py --workload chr22 --cpu-seconds 5
cd /tmp
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline
exit 0
