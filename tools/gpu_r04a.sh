# round 4: new request_eval_kernel (64 chains per run, chain lookup by
# readlane + mbcnt, per-chain sums by DPP scans) -- request tests, config 3
# bench + kernel trace; then the round-3 64-slot kernel with bounds checks
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04a}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.log | cut -c1-600
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 400 python3 -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread -k "requests or genome or chains"
step genome 600 python3 -u $R/bench.py --no-cpu-baseline
cd /tmp
step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline
cd $R
SBEACON_LIB=$R/tools/r64/libsbeacon_hip_r64.so step r64 300 python3 -u -m pytest $R/tests/test_gpu_requests.py -x -v -s --timeout 120 --timeout-method thread -k "genome_requests_match"
exit 0
