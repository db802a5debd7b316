# round-3 validation B: config 5 (gnomAD shape) and config 4 (50 datasets: summarise, dedup, strict dedup)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r03B}
mkdir -p $OUT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; grep '^{' $OUT/$name.log | cut -c1-300; tail -1 $OUT/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step paths 900 python3 -u $R/bench_paths.py --datasets 50 --steps 10 --warmup 2
step gnomad 1000 python3 -u $R/bench.py --workload gnomad --steps 10 --warmup 2
exit 0
