# round 4: SQ counters of the new request_eval_kernel (reduced config 3:
# 20 M records, 250 k requests -- the same per-wave shape), then the round-3
# 64-slot kernel with bounds checks on the faulting test
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04b}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.log | cut -c1-400
  case $rc in 0) return 0;; *) exit $rc;; esac
}
GA="--genome-records 20000000 --genome-requests 250000 --steps 2 --warmup 1 --no-cpu-baseline"
cd /tmp
step sq1 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d $OUT/sq1 -o run -- python3 $R/bench.py $GA
step sq2 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_INSTS_SMEM --kernel-trace --output-format csv -d $OUT/sq2 -o run -- python3 $R/bench.py $GA
step sq3 300 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SALU --kernel-trace --output-format csv -d $OUT/sq3 -o run -- python3 $R/bench.py $GA
cd $R
python3 tools/sq_summary.py $OUT/sq1 $OUT/sq2 $OUT/sq3 > $OUT/sq_summary.txt 2>&1; grep -A0 "request_eval" $OUT/sq_summary.txt | cut -c1-600
SBEACON_LIB=$R/tools/r64/libsbeacon_hip_r64.so step r64 300 python3 -u -m pytest $R/tests/test_gpu_requests.py -x -v -s --timeout 120 --timeout-method thread -k "genome_requests_match"
exit 0
