TAG=r06s5
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 1 $O/$name.log | cut -c1-1500; case $rc in 0) return 0;; *) exit $rc;; esac; }
step bench 500 python3 -u $R/bench.py --steps 20 --warmup 5 --no-config4 --no-config5 --no-config2 --no-cpu-baseline
cd /tmp
step prof 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 -u $R/bench.py --steps 20 --warmup 5 --no-config4 --no-config5 --no-config2 --no-cpu-baseline
exit 0
