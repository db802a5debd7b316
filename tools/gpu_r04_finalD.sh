# round-4 final B (second pass) + config 5: config 4 (dedup, summarise, strict) + its PMC traffic, config 2 (wire)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04GB}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.log | cut -c1-400
  case $rc in 0) return 0;; *) exit $rc;; esac
}
SBEACON_DEDUP_DEBUG=1 step paths 700 python3 -u $R/bench_paths.py --datasets 50
cd /tmp
GA="--datasets 50 --steps 2 --warmup 1 --no-cpu-baseline --strict-datasets 0"
step pfetch 500 timeout -s KILL 490 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_pfetch -o run -- python3 $R/bench_paths.py $GA
step pwrite 500 timeout -s KILL 490 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_pwrite -o run -- python3 $R/bench_paths.py $GA
cd $R && python3 tools/pmc_traffic.py $OUT/pmc_pfetch $OUT/pmc_pwrite --records 110354700 --requests 50 --out $OUT/traffic_paths.json > /dev/null && echo folded paths
step chr22 500 python3 -u $R/bench.py --workload chr22 --cpu-seconds 8
SBEACON_WIRE_TRACE=1 step wire 300 python3 -u $R/tools/wire_split.py

step gnomad 700 python3 -u $R/bench.py --workload gnomad
exit 0
