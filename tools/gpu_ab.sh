# A/B of library variants on the config-3 request pass (tools/req_tune.py,
# 4 rotating 1 M-request batches re-planned each pass, compact outputs):
# the store is built and saved once, each variant re-opens it; VARIANTS =
# names under tools/variants/ (tools/build_variant.sh).  SQ = variants whose
# SQ instruction counters are collected (one rocprofv3 pass each).  Outputs
# under gpurun_out/$TAG; stops at the first failure.
TAG=${TAG:-ab}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -n 1 $O/$name.log | cut -c1-400
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step save 400 python3 -u $R/tools/req_tune.py --save /tmp/st --rounds 2
i=0
for v in $VARIANTS; do  # (ab_<variant>_<i>.log: a variant listed twice keeps both runs)
  i=$((i+1))
  SBEACON_LIB=$R/tools/variants/$v/libsbeacon_hip.so step ab_${v}_$i 200 python3 -u $R/tools/req_tune.py --open /tmp/st --rounds ${ROUNDS:-15} --digest
done
for v in $SQ; do  # SQ = variants whose SQ instruction counters are collected (one rocprofv3 pass each)
  ( cd /tmp && SBEACON_LIB=$R/tools/variants/$v/libsbeacon_hip.so step sq_$v 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/sq_$v -o p -- python3 -u $R/tools/req_tune.py --open /tmp/st --rounds 2 ) || exit 1
done
exit 0
