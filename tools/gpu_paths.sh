# dedup/summarise GPU tests -> bench_paths (summarise + dedup, config 4) -> rocprofv3 kernel trace of it
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
DS=${DS:-10}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -6 $R/gpurun_out/$name.log
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step gpu_tests_paths 600 python3 -u -m pytest tests/test_gpu_dedup.py tests/test_gpu_summarise.py -m gpu -x -v --timeout 300 --timeout-method thread
step paths 900 python3 -u $R/bench_paths.py --datasets $DS
cd /tmp && step paths_prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/paths_prof -o paths -- python3 $R/bench_paths.py --datasets $DS --steps 5 --no-cpu-baseline
exit 0
