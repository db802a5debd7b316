# wire in-place writes + genotype bit-matrix config-3 store: tests, wire split, default bench
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04y}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 600 python3 -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread -k "wire or genome or beacon or requests or parity"
SBEACON_WIRE_TRACE=1 step wire 300 python3 -u $R/tools/wire_split.py
step wire_plain 300 python3 -u $R/tools/wire_split.py
step genome 700 python3 -u $R/bench.py
exit 0
