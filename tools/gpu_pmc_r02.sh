# PMC HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes, kernel trace
# only) for the round-2 bench lines: config 3 (chain_pack_kernel<false>) and
# config 4 (summarise + window dedup kernels), folded by tools/pmc_traffic.py
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 $R/gpurun_out/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
cd /tmp
if [ -z "${NO_GENOME:-}" ]; then
GA="--workload genome --steps 2 --warmup 1 --no-cpu-baseline"
step pmc_fetch_g 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch_g -o run -- python3 $R/bench.py $GA
step pmc_write_g 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write_g -o run -- python3 $R/bench.py $GA
(cd $R && python3 tools/pmc_traffic.py gpurun_out/pmc_fetch_g gpurun_out/pmc_write_g --records 85000000 --requests 1000000 --kernel 'chain_pack_kernel<false>' --out gpurun_out/traffic_genome.json > /dev/null && echo folded genome)
fi
PA="--datasets 50 --steps 2 --warmup 1 --no-cpu-baseline"
step pmc_fetch_p 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch_p -o run -- python3 $R/bench_paths.py $PA
step pmc_write_p 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write_p -o run -- python3 $R/bench_paths.py $PA
(cd $R && python3 tools/pmc_traffic.py gpurun_out/pmc_fetch_p gpurun_out/pmc_write_p --records 110354700 --requests 50 --out gpurun_out/traffic_paths.json > /dev/null && echo folded paths)
exit 0
