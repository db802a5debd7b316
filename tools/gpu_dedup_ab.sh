# config-4 dedup (tools/dedup_ablate.py): window-kernel timings and counts
# of the in-tree library and of each variant in $VARIANTS
mkdir -p gpurun_out/${TAG:-gpu_dedup_ab}
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-gpu_dedup_ab}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; grep -a "mode" $O/$name.log | cut -c1-200
  case $rc in 0) return 0;; *) exit $rc;; esac
}
V=$R/tools/variants
step base 400 python3 -u $R/tools/dedup_ablate.py --save /tmp/dst --modes ${MODES:-0,1,0}
for v in $VARIANTS; do
  step $v 200 env SBEACON_LIB=$V/$v/libsbeacon_hip.so python3 -u $R/tools/dedup_ablate.py --open /tmp/dst --modes ${MODES:-0,1,0}
done
exit 0
