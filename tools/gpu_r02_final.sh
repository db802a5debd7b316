# Round-2 refresh: config 2 and config 5 bench lines, config-3 PMC traffic of
# the current chain kernel (FETCH / WRITE passes), window-dedup kernel trace
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r02_final}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -1 $OUT/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step chr22 600 python3 -u $R/bench.py --workload chr22 --steps 20 --warmup 3
step gnomad 900 python3 -u $R/bench.py --workload gnomad --steps 10 --warmup 2
cd /tmp
GA="--workload genome --steps 2 --warmup 1 --no-cpu-baseline"
step pmc_fetch_g 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch_g -o run -- python3 $R/bench.py $GA
step pmc_write_g 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write_g -o run -- python3 $R/bench.py $GA
(cd $R && python3 tools/pmc_traffic.py $OUT/pmc_fetch_g $OUT/pmc_write_g --records 85000000 --requests 1000000 --kernel 'chain_pack_kernel<false>' --out $OUT/traffic_genome.json > /dev/null && echo folded genome)
step dedup_prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/dedup_prof -o run -- python3 $R/bench_paths.py --datasets 50 --only dedup --steps 5 --warmup 1 --no-cpu-baseline
exit 0
