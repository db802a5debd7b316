# Config 5 (bench.py --workload gnomad) with the per-slice batch's second
# stream created CU-masked (in-tree library) against a plain one (the HEAD
# build under tools/variants/head), then every GPU test on the in-tree
# library.  Outputs under gpurun_out/$TAG.
TAG=${TAG:-aux}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 1 $O/$name.log | cut -c1-400; case $rc in 0) return 0;; *) exit $rc;; esac; }
step g_new1 300 python3 -u $R/bench.py --workload gnomad --steps 20 --warmup 5 --no-cpu-baseline
SBEACON_LIB=$R/tools/variants/head/libsbeacon_hip.so step g_head 300 python3 -u $R/bench.py --workload gnomad --steps 20 --warmup 5 --no-cpu-baseline
step g_new2 300 python3 -u $R/bench.py --workload gnomad --steps 20 --warmup 5 --no-cpu-baseline
step gpu_tests 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
exit 0
