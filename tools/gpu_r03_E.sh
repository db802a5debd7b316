# request tests at both run sizes + config 3 A/B: 32 vs 64 chain slots per run
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r03E}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; grep '^{' $OUT/$name.log | cut -c1-250; tail -1 $OUT/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 300 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread -k "requests or genome"
step genome 600 python3 -u $R/bench.py --no-cpu-baseline
SBEACON_WIRE_TRACE=1 step wire 300 python3 -u $R/tools/wire_split.py
exit 0
