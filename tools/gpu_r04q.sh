# wire path with the per-store variant text cache: wire tests + config-2 split
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04q}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 400 python3 -u -m pytest $R/tests/test_gpu_wire.py -x -v --timeout 120 --timeout-method thread
step wire_plain 400 python3 -u $R/tools/wire_split.py
SBEACON_WIRE_TRACE=1 step wire 400 python3 -u $R/tools/wire_split.py
grep "\[wire\]\|\[query\]\|\[prepare\]" $OUT/wire.log | tail -16
grep call_ms $OUT/wire_plain.log
exit 0
