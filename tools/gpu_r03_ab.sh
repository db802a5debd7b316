# request-path A/B + request tests + config-3 bench (prepare trace on)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r03ab}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.log | cut -c1-600
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 300 python3 -u -m pytest $R/tests/test_gpu_requests.py -x -v --timeout 120 --timeout-method thread
step ab 500 python3 -u $R/tools/req_ab.py
SBEACON_PREP_TRACE=1 step bench 600 python3 -u $R/bench.py --no-cpu-baseline
exit 0
