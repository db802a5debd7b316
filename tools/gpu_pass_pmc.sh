# memory-side counters of the request pass (TCP / UTCL1 / TCC / TA / TD / GRBM), one pass each
mkdir -p gpurun_out/${TAG:-gpu_pass_pmc}
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-gpu_pass_pmc}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
cd /tmp
step save 300 python3 -u $R/tools/req_tune.py --save /tmp/st --rounds 3
P() { local n=$1; shift; step pmc_$n 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/pmc_$n -o p -- python3 -u $R/tools/req_tune.py --open /tmp/st --rounds 2; }
P a TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum
P b TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum
P c TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum
P d TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY
P e TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCR_TCP_STALL_CYCLES_sum
exit 0
