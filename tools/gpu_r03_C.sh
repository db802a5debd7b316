# request tests (32 B request descriptors, pooled buffers) + config 3 with host
# planning phase times + validation B (config 4 with strict mode, config 5)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r03C}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; grep '^{' $OUT/$name.log | cut -c1-300; tail -1 $OUT/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 300 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread -k "requests or genome or wire"
SBEACON_PREP_TRACE=1 step genome 600 python3 -u $R/bench.py --no-cpu-baseline
SBEACON_WIRE_TRACE=1 step wire 300 python3 -u $R/tools/wire_split.py
step paths 900 python3 -u $R/bench_paths.py --datasets 50 --steps 10 --warmup 2 --strict-datasets 3
step gnomad 900 python3 -u $R/bench.py --workload gnomad --steps 10 --warmup 2
exit 0
