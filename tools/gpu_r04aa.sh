# async fan-in + handler parity on the device, then the config-2 bench line
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04aa}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 500 python3 -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread -k "variant_queries or parity or route"
step chr22 500 python3 -u $R/bench.py --workload chr22 --cpu-seconds 8
exit 0
