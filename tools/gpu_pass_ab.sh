# request pass on 4 rotating 1 M batches (tools/req_tune.py): eval / pass
# timing and the outputs' digest of the in-tree library, then of every
# library variant named in $VARIANTS (tools/build_variant.sh NAME ...)
mkdir -p gpurun_out/${TAG:-gpu_pass_ab}
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-gpu_pass_ab}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-400
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step full 300 python3 -u $R/tools/req_tune.py --save /tmp/st --digest
for v in $VARIANTS; do
  step $v 200 env SBEACON_LIB=$R/tools/variants/$v/libsbeacon_hip.so python3 -u $R/tools/req_tune.py --open /tmp/st --digest
done
exit 0
