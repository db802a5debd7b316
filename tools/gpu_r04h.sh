# round 4: window kernel with incremental piece walk + persisted-store open
# with mapped host.bin (columns loaded beside the device image)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04h}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 400 python3 -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread -k "dedup or pipeline or persist"
SBEACON_DEDUP_DEBUG=1 step paths 600 python3 -u $R/bench_paths.py --datasets 50 --only dedup --no-cpu-baseline
grep "dedup:\|strict:" $OUT/paths.log
cd /tmp
step dsq1 500 timeout -s KILL 490 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d $OUT/dsq1 -o run -- python3 $R/bench_paths.py --datasets 50 --only dedup --steps 2 --warmup 1 --no-cpu-baseline --strict-datasets 0
cd $R
python3 tools/sq_summary.py $OUT/dsq1 > $OUT/dsq_summary.txt 2>&1; grep "window_dedupe" $OUT/dsq_summary.txt | cut -c1-400
step persist 600 python3 -u tools/persist_bench.py
tail -1 $OUT/persist.log
SBEACON_PREP_TRACE=1 step genome 600 python3 -u $R/bench.py --no-cpu-baseline
grep -o '"delivered[^}]*}[^}]*}' $OUT/genome.log
exit 0
