# round 5: eval-kernel A/B (pre-change library vs in-tree) + SQ counters of the in-tree pass
mkdir -p gpurun_out/r05c
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05c
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-400
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step new 300 python3 -u $R/tools/req_tune.py --save /tmp/st --digest
step base 300 env SBEACON_LIB=$R/tools/variants/r05base/libsbeacon_hip.so python3 -u $R/tools/req_tune.py --digest
step new2 200 python3 -u $R/tools/req_tune.py --open /tmp/st --digest
cd /tmp
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
C2="SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_BUSY_CYCLES"
step pmc1 200 rocprofv3 --pmc $C1 --kernel-trace --output-format csv -d $O/pmc1 -o p -- python3 -u $R/tools/req_tune.py --open /tmp/st --rounds 3
step pmc2 200 rocprofv3 --pmc $C2 --kernel-trace --output-format csv -d $O/pmc2 -o p -- python3 -u $R/tools/req_tune.py --open /tmp/st --rounds 3
exit 0
