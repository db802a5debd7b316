# round-4 final E: smoke, every GPU test, config 3 (default bench line, carrier bit-matrix store)
# + kernel trace + PMC traffic of request_eval_kernel, config 2 (step + wire)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04FE}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.log | cut -c1-400
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()"
step tests 700 python3 -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread
step genome 600 python3 -u $R/bench.py
step chr22 500 python3 -u $R/bench.py --workload chr22 --cpu-seconds 8
cd /tmp
step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline
GA="--steps 2 --warmup 1 --no-cpu-baseline"
step fetch 400 timeout -s KILL 390 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $GA
step write 400 timeout -s KILL 390 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py $GA
cd $R && python3 tools/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write --records 85000000 --requests 1000000 --kernel request_eval_kernel --out $OUT/traffic_genome.json > /dev/null && echo folded
exit 0
