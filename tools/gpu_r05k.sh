# round 5: window_dedupe_kernel with identities in registers -- dedup GPU tests, config-4
# timings (modes 0 / 4 loads only / 1 no rounds) against the round-4 kernel
# (variant old) and a 5-waves build (s8k: 8192 slots), kernel stats
mkdir -p gpurun_out/r05k
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05k
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-300
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dedup.py tests/test_gpu_pipeline.py
step new 400 python3 -u $R/tools/dedup_ablate.py --save /tmp/dst --modes 0,4,1,0
step old 200 env SBEACON_LIB=$R/tools/variants/old/libsbeacon_hip.so python3 -u $R/tools/dedup_ablate.py --open /tmp/dst --modes 0,4,1,0
step s8k 200 env SBEACON_LIB=$R/tools/variants/s8k/libsbeacon_hip.so python3 -u $R/tools/dedup_ablate.py --open /tmp/dst --modes 0,1,0
cd /tmp
step prof 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u $R/tools/dedup_ablate.py --open /tmp/dst --modes 0
exit 0
