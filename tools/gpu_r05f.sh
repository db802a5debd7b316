# round 5: request-path GPU tests + A/B of the in-tree pass vs a variant library
mkdir -p gpurun_out/r05f
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05f
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-400
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "requests or genome or persist or beacon or chains"
step new 300 python3 -u $R/tools/req_tune.py --digest
for v in $VARIANTS; do
  step $v 300 env SBEACON_LIB=$R/tools/variants/$v/libsbeacon_hip.so python3 -u $R/tools/req_tune.py --digest
done
exit 0
