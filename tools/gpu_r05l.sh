# round 5: persistent window_dedupe_kernel diagnosis -- grid size from the
# occupancy query (SBEACON_DEDUP_DEBUG prints it) vs forced grids, 6 / 5 waves
mkdir -p gpurun_out/r05l
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05l
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; grep -a "mode\|window kernel" $O/$name.log | sort | uniq -c | cut -c1-200
  case $rc in 0) return 0;; *) exit $rc;; esac
}
V=$R/tools/variants
step new 400 python3 -u $R/tools/dedup_ablate.py --save /tmp/dst --modes 0,4,0
step p6 200 env SBEACON_DEDUP_DEBUG=1 SBEACON_LIB=$V/pers6/libsbeacon_hip.so python3 -u $R/tools/dedup_ablate.py --open /tmp/dst --modes 0,4
step p6g1536 200 env SBEACON_DEDUP_WIN_GRID=1536 SBEACON_LIB=$V/pers6/libsbeacon_hip.so python3 -u $R/tools/dedup_ablate.py --open /tmp/dst --modes 0,4
step p6g3072 200 env SBEACON_DEDUP_WIN_GRID=3072 SBEACON_LIB=$V/pers6/libsbeacon_hip.so python3 -u $R/tools/dedup_ablate.py --open /tmp/dst --modes 0,4
step p5 200 env SBEACON_DEDUP_DEBUG=1 SBEACON_LIB=$V/pers5/libsbeacon_hip.so python3 -u $R/tools/dedup_ablate.py --open /tmp/dst --modes 0,4
exit 0
