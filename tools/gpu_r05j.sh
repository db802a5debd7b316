# round 5: every GPU test + smoke (validation of the round's changes)
mkdir -p gpurun_out/r05j
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05j
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step tests 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread
exit 0
