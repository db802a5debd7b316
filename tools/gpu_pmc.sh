# PMC passes (FETCH_SIZE, then WRITE_SIZE — they do not fit one pass on
# gfx950) over a short bench run, kernel trace only; then fold into
# profiles/traffic.json.  No sys/runtime traces with --pmc.
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 $R/gpurun_out/$name.log
  case $rc in 0|1) return 0;; *) exit $rc;; esac
}
cd /tmp
step pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline
step pmc_write 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline
cd $R && python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --out gpurun_out/traffic.json
exit 0
