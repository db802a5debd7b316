# dedup: GPU tests, config-4 dedup bench (50 datasets) + kernel trace, PMC traffic of the window kernel
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r03dd}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; grep '^{' $OUT/$name.log | cut -c1-300; tail -2 $OUT/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 400 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread -k "dedup or pipeline or wire"
SBEACON_WIRE_TRACE=1 step wire 300 python3 -u $R/tools/wire_split.py
step paths 900 python3 -u $R/bench_paths.py --datasets 50 --only dedup --steps 10 --warmup 2 --no-cpu-baseline
cd /tmp
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench_paths.py --datasets 50 --only dedup --steps 5 --warmup 1 --no-cpu-baseline
step fetch 550 timeout -s KILL 540 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench_paths.py --datasets 50 --only dedup --steps 2 --warmup 1 --no-cpu-baseline
exit 0
