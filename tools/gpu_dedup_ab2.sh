# window dedup timing ablations (SBEACON_DEDUP_WIN_DBG bits: 1 no exact inserts, 2 no hashed inserts, 4 loads only)
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=${D:-10}
for dbg in 0 1 2 3 4; do
  SBEACON_DEDUP_WIN_DBG=$dbg timeout -k 10 300 python3 -u $R/bench_paths.py --datasets $D --only dedup --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/ab2_$dbg.log 2>&1 || exit 1
  echo "dbg=$dbg $(grep -o 'device_ms_per_step\": [0-9.]*' $R/gpurun_out/ab2_$dbg.log | tail -1)"
done
