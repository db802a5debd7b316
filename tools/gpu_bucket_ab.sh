# Smoke + every GPU test, then an A/B of the coarse candidate index's bucket
# size (SBEACON_VC_BUCKET, read when the store is built): the config-3
# request pass (tools/req_tune.py, 4 rotating 1 M batches, digests) on a
# store built with each setting.  Outputs under gpurun_out/$TAG.
TAG=${TAG:-bucket}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -n 1 $O/$name.log | cut -c1-600
  case $rc in 0) return 0;; *) exit $rc;; esac
}
${SKIP_TESTS:+false} step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" || true
${SKIP_TESTS:+false} step gpu_tests 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread || true
i=0
for b in ${BUCKETS:-1.0 0.5 0.25 1.0}; do
  i=$((i+1))
  SBEACON_VC_BUCKET=$b step vcb_${i}_$b 300 python3 -u $R/tools/req_tune.py --rounds ${ROUNDS:-15} --digest
done
exit 0
