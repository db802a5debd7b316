# round-end validation: smoke, every GPU test, the three bench lines
# (config 2 default, config 3 genome, config 5 gnomad) and a rocprofv3
# kernel summary of each bench command; stops at the first failure
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 $R/gpurun_out/$name.log | cut -c1-400
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread
step bench 300 python3 -u $R/bench.py --steps 20 --warmup 3
step genome 300 python3 -u $R/bench.py --workload genome --steps 5 --warmup 1
step gnomad 300 python3 -u $R/bench.py --workload gnomad --steps 20 --warmup 3
cd /tmp
step prof_bench 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fprof -o bench -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline
step prof_genome 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fprof -o genome -- python3 $R/bench.py --workload genome --steps 5 --warmup 1 --no-cpu-baseline
step prof_gnomad 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fprof -o gnomad -- python3 $R/bench.py --workload gnomad --steps 20 --warmup 3 --no-cpu-baseline
exit 0
