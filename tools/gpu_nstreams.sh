# Config-3 step with 1-4 batches in flight (--streams N, CU-masked streams).
# Outputs under gpurun_out/$TAG.
TAG=${TAG:-nstreams}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep '^{' $O/$name.log | tail -n 1 | cut -c1-260; case $rc in 0) return 0;; *) exit $rc;; esac; }
for n in ${NS:-2 3 4}; do
  step s_$n 400 python3 -u $R/bench.py --steps 40 --warmup 5 --no-config4 --no-config5 --no-config2 --no-cpu-baseline --streams $n
done
exit 0
