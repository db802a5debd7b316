# rocprofv3 kernel summaries of the config-5 and config-2 lines with two
# copies of the batch in flight (bench.py --workload gnomad / chr22).
TAG=${TAG:-profsubs}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep '^{' $O/$name.log | tail -n 1 | cut -c1-200; case $rc in 0) return 0;; *) exit $rc;; esac; }
cd /tmp
step prof_gnomad 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gnomad -o g -- python3 -u $R/bench.py --workload gnomad --steps 20 --warmup 5 --no-cpu-baseline
step prof_chr22 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/chr22 -o c -- python3 -u $R/bench.py --workload chr22 --steps 20 --warmup 5 --no-cpu-baseline
exit 0
