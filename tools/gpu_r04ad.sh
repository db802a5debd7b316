# sanity on the final in-tree library: smoke + request / genome / wire tests
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04ad}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()"
step tests 600 python3 -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread
exit 0
