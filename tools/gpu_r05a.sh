# round 5: copy-engine probe, the GPU tests touched this round, the config-3
# bench (rotating batches, planning inside the step) and its kernel trace
mkdir -p gpurun_out/r05a
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05a
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-600
  case $rc in 0) return 0;; *) exit $rc;; esac
}
env | grep -iE '^(HSA|HIP|GPU|ROC|AMD)_' > $O/env.txt
nproc > $O/cpus.txt; python3 -c "import os; print(len(os.sched_getaffinity(0)))" >> $O/cpus.txt; cat /sys/fs/cgroup/cpu.max >> $O/cpus.txt 2>&1; lscpu | grep -i 'model name' >> $O/cpus.txt
step tests 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "dedup or pipeline or requests or genome"
cd /tmp
step probe_default 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/probe_default -o p -- python3 $R/tools/copy_probe.py
step genome 600 python3 -u $R/bench.py --steps 20 --warmup 5
step genome_prof 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/genome -o g -- python3 -u $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline
exit 0
