# config 5: bench at full size, then FETCH_SIZE / WRITE_SIZE passes (kernel
# trace only, separate runs) folded into gpurun_out/traffic_gnomad.json
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 $R/gpurun_out/$name.log
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step gnomad_full 600 python3 -u $R/bench.py --workload gnomad --steps 20 --warmup 3
cd /tmp
step pmc_fetch_g 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch_g -o run -- python3 $R/bench.py --workload gnomad --steps 5 --warmup 1 --no-cpu-baseline
step pmc_write_g 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write_g -o run -- python3 $R/bench.py --workload gnomad --steps 5 --warmup 1 --no-cpu-baseline
cd $R && python3 tools/pmc_traffic.py gpurun_out/pmc_fetch_g gpurun_out/pmc_write_g --records 750000000 --requests 50000 --out gpurun_out/traffic_gnomad.json > /dev/null && echo folded
exit 0
