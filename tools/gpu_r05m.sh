# round 5: window_dedupe_kernel slot-set size / LDS footprint (7 workgroups
# per CU at <= 23 KB) -- config-4 timings and counts per variant
mkdir -p gpurun_out/r05m
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05m
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; grep -a "mode" $O/$name.log | cut -c1-200
  case $rc in 0) return 0;; *) exit $rc;; esac
}
V=$R/tools/variants
step base 400 python3 -u $R/tools/dedup_ablate.py --save /tmp/dst --modes 0,1,0
for v in s3072 s2816 s2048; do
  step $v 200 env SBEACON_LIB=$V/$v/libsbeacon_hip.so python3 -u $R/tools/dedup_ablate.py --open /tmp/dst --modes 0,1,0
done
exit 0
