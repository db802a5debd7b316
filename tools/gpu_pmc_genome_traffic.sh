# config 3: FETCH_SIZE / WRITE_SIZE passes (kernel trace only, separate runs)
# over the genome bench, folded into gpurun_out/traffic_genome.json
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
ARGS="--workload genome --steps 2 --warmup 1 --no-cpu-baseline"
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -2 $R/gpurun_out/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
cd /tmp
step pmc_fetch_w 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch_w -o run -- python3 $R/bench.py $ARGS
step pmc_write_w 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write_w -o run -- python3 $R/bench.py $ARGS
cd $R && python3 tools/pmc_traffic.py gpurun_out/pmc_fetch_w gpurun_out/pmc_write_w --records 85000000 --requests 1000000 --kernel chain_kernel --out gpurun_out/traffic_genome.json > /dev/null && echo folded
exit 0
