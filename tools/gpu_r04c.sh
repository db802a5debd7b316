# round 4: request_eval_kernel counters on the FULL config 3 (85 M records,
# 1 M requests): SQ issue/wait, L2 hit/miss; plus the counter list
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04c}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
GA="--steps 2 --warmup 1 --no-cpu-baseline"
cd /tmp
step list 60 rocprofv3 -L
step sq1 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d $OUT/sq1 -o run -- python3 $R/bench.py $GA
step tcc 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --kernel-trace --output-format csv -d $OUT/tcc -o run -- python3 $R/bench.py $GA
cd $R
python3 tools/sq_summary.py $OUT/sq1 $OUT/tcc > $OUT/sq_summary.txt 2>&1; grep "request_eval" $OUT/sq_summary.txt | cut -c1-600
exit 0
