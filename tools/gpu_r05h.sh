# round 5: the default bench line (config 3) + its kernel trace
mkdir -p gpurun_out/r05h
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05h
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
cd /tmp
step genome 600 python3 -u $R/bench.py --steps 20 --warmup 5

exit 0
