# round 5: coarse candidate index granularity (SBEACON_VC_BUCKET) A/B + kernel trace of the pass
mkdir -p gpurun_out/r05g
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05g
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-400
  case $rc in 0) return 0;; *) exit $rc;; esac
}
cd /tmp
step b1 300 python3 -u $R/tools/req_tune.py --digest
step b05 300 env SBEACON_VC_BUCKET=0.5 python3 -u $R/tools/req_tune.py --digest
exit 0
