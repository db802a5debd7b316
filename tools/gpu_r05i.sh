# round 5: host preparation phases of a request batch + the async fan-in / dedup GPU tests
mkdir -p gpurun_out/r05i
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05i
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "variant_queries or dedup or pipeline"
step prep 300 env SBEACON_PREP_TRACE=1 python3 -u $R/tools/prep_trace.py
exit 0
