# round 4: device request planning (request_plan_kernel) -- request tests,
# the default bench line (config 3, delivered path), then SQ counters of the
# full config
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04d}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 400 python3 -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread -k "requests or genome or chains"
SBEACON_PREP_TRACE=1 step genome 600 python3 -u $R/bench.py
GA="--steps 2 --warmup 1 --no-cpu-baseline"
cd /tmp
step sq1 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d $OUT/sq1 -o run -- python3 $R/bench.py $GA
cd $R
python3 tools/sq_summary.py $OUT/sq1 > $OUT/sq_summary.txt 2>&1; grep "request_eval\|request_plan" $OUT/sq_summary.txt | cut -c1-600
exit 0
