# dedup tests + config 4 (window planning split into POS-range tasks; plan times under SBEACON_DEDUP_DEBUG)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r03I}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; grep '^{' $OUT/$name.log | cut -c1-250; tail -1 $OUT/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 400 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread -k "dedup or pipeline"
SBEACON_DEDUP_DEBUG=1 step paths 900 python3 -u $R/bench_paths.py --datasets 50 --steps 10 --warmup 2 --strict-datasets 10
exit 0
