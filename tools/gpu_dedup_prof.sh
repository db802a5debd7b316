# dedup only (config-4 shape, D datasets): window path, bucket path, kernel trace
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-dprof}
mkdir -p $OUT
D=${D:-10}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -1 $OUT/$name.log | cut -c1-900
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step win 400 python3 -u $R/bench_paths.py --datasets $D --only dedup --steps 5 --warmup 1 --no-cpu-baseline
cd /tmp && step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench_paths.py --datasets $D --only dedup --steps 5 --warmup 1 --no-cpu-baseline
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
cut -d, -f1-4 $OUT/kernel_stats.csv | cut -c1-160 | head -14
exit 0
