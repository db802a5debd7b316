# window dedup: GPU dedup tests, then config 4 (50 datasets) bench
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-win}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -4 $OUT/$name.log | cut -c1-1500
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 600 python3 -u -m pytest tests/test_gpu_dedup.py ${EXTRA_TESTS:-} -m gpu -x -v --timeout 200 --timeout-method thread
step paths 600 python3 -u $R/bench_paths.py --datasets 50 --steps 10 --warmup 2
exit 0
