# round 5: request-path GPU tests + the config-3 bench + its kernel trace
mkdir -p gpurun_out/r05b
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05b
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-600
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "requests or genome or persist or beacon or chains"
cd /tmp
step genome 600 python3 -u $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline
step genome_prof 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/genome -o g -- python3 -u $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline
exit 0
