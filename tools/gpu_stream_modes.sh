# Which stream creation puts the bench step's two streams on separate
# hardware queues (SBEACON_BENCH_STREAMS: prio / cumask / plain; --streams 1
# beside them)?  Config 3 only, no CPU baseline.  Outputs under gpurun_out/$TAG.
TAG=${TAG:-smodes}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 1 $O/$name.log | cut -c1-300; case $rc in 0) return 0;; *) exit $rc;; esac; }
for m in ${MODES:-prio cumask plain}; do
  SBEACON_BENCH_STREAMS=$m step b_$m 400 python3 -u $R/bench.py --steps 40 --warmup 5 --no-config4 --no-config5 --no-config2 --no-cpu-baseline
done
step b_one 400 python3 -u $R/bench.py --steps 40 --warmup 5 --no-config4 --no-config5 --no-config2 --no-cpu-baseline --streams 1
exit 0
