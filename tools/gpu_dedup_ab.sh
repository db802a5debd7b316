# dedup A/B at config 4 (50 datasets): bucket path, bucket without inserts (timing only), radix path
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
for mode in bucket nobody radix; do
  case $mode in
    bucket) env_="";;
    nobody) env_="SBEACON_DEDUP_BUCKET_DBG=1";;
    radix) env_="SBEACON_DEDUP_EXACT=radix";;
  esac
  env $env_ timeout -k 10 300 python3 -u $R/bench_paths.py --datasets 50 --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/ab_$mode.log 2>&1 || exit 1
  echo "$mode $(grep -o 'device_ms_per_step\": [0-9.]*' $R/gpurun_out/ab_$mode.log | tail -1)"
done
