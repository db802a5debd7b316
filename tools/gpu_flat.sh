# flattened sample path: the 2,504-sample parity test first, then every GPU
# test, smoke, the config-5 bench and its rocprofv3 kernel summary
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 $R/gpurun_out/$name.log | cut -c1-600
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step flat_test 200 python3 -u -m pytest tests/test_gnomad.py -m gpu -x -v --timeout 120 --timeout-method thread
step gpu_tests 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step gnomad 300 python3 -u $R/bench.py --workload gnomad --steps 20 --warmup 3
cd /tmp
step prof_gnomad 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fprof -o gnomad -- python3 $R/bench.py --workload gnomad --steps 20 --warmup 3 --no-cpu-baseline
exit 0
