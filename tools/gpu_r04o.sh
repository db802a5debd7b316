# SQ counters of the window dedup kernel (config 4, 50 datasets)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04o}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -1 $OUT/$name.log | cut -c1-200
  case $rc in 0) return 0;; *) exit $rc;; esac
}
cd /tmp
step dsq1 400 timeout -s KILL 390 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d $OUT/dsq1 -o run -- python3 $R/bench_paths.py --datasets 50 --only dedup --steps 2 --warmup 1 --no-cpu-baseline --strict-datasets 0
step dsq2 400 timeout -s KILL 390 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $OUT/dsq2 -o run -- python3 $R/bench_paths.py --datasets 50 --only dedup --steps 2 --warmup 1 --no-cpu-baseline --strict-datasets 0
cd $R
python3 tools/sq_summary.py $OUT/dsq1 $OUT/dsq2 > $OUT/dsq_summary.txt 2>&1; grep "window_dedupe" $OUT/dsq_summary.txt | cut -c1-500
exit 0
