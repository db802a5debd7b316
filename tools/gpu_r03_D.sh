# request / wire / dedup tests, config 3 (planning phase times), config-2 wire
# split, config 4 (strict dedup with cached region files), PMC passes of
# request_eval_kernel (32 B descriptors)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r03D}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; grep '^{' $OUT/$name.log | cut -c1-300; tail -1 $OUT/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 400 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread -k "requests or genome or wire or pipeline or dedup"
SBEACON_PREP_TRACE=1 step genome 600 python3 -u $R/bench.py --no-cpu-baseline
SBEACON_WIRE_TRACE=1 step wire 300 python3 -u $R/tools/wire_split.py
step paths 900 python3 -u $R/bench_paths.py --datasets 50 --steps 10 --warmup 2 --strict-datasets 10
cd /tmp
GA="--steps 2 --warmup 1 --no-cpu-baseline"
step fetch 400 timeout -s KILL 390 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $GA
step write 400 timeout -s KILL 390 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py $GA
cd $R && python3 tools/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write --records 85000000 --requests 1000000 --kernel request_eval_kernel --out $OUT/traffic_genome.json > /dev/null && echo folded
exit 0
