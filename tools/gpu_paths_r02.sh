# config 4 at BASELINE's 50 datasets x 2 VCFs: the two bench lines
# (PMC=1: FETCH_SIZE / WRITE_SIZE passes instead, folded into traffic_paths.json)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
DS=${DS:-50}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; grep '^{' $R/gpurun_out/$name.log | cut -c1-400; tail -2 $R/gpurun_out/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
if [ -z "${PMC:-}" ]; then
  step paths_bench 1000 python3 -u $R/bench_paths.py --datasets $DS --steps 10 --warmup 2
else
  cd /tmp
  step paths_fetch 550 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_paths_fetch -o run -- python3 $R/bench_paths.py --datasets $DS --steps 2 --warmup 1 --no-cpu-baseline
  step paths_write 550 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_paths_write -o run -- python3 $R/bench_paths.py --datasets $DS --steps 2 --warmup 1 --no-cpu-baseline
  cd $R && python3 tools/pmc_traffic.py gpurun_out/pmc_paths_fetch gpurun_out/pmc_paths_write --records 0 --requests 0 --out gpurun_out/traffic_paths.json > /dev/null && echo folded
fi
exit 0
