# Config 5 (bench.py --workload gnomad) one batch at a time against two
# copies in flight on CU-masked streams; the last run with the CPU baseline
# and the oracle parity sample.  Outputs under gpurun_out/$TAG.
TAG=${TAG:-gnomads}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep '^{' $O/$name.log | tail -n 1 | cut -c1-300; case $rc in 0) return 0;; *) exit $rc;; esac; }
step c_1 300 python3 -u $R/bench.py --workload gnomad --steps 40 --warmup 5 --no-cpu-baseline --streams 1
step c_2 300 python3 -u $R/bench.py --workload gnomad --steps 40 --warmup 5 --no-cpu-baseline --streams 2
step c_1b 300 python3 -u $R/bench.py --workload gnomad --steps 40 --warmup 5 --no-cpu-baseline --streams 1
step c_2full 300 python3 -u $R/bench.py --workload gnomad --steps 20 --warmup 5
exit 0
