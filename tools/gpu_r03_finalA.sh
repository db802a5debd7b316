# round-3 validation A: smoke, every GPU test, config 3 (default bench line) + kernel trace, config 2
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r03A}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.log | cut -c1-400
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()"
step tests 600 python3 -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread
step genome 600 python3 -u $R/bench.py
step chr22 400 python3 -u $R/bench.py --workload chr22 --cpu-seconds 8
cd /tmp
step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline
exit 0
