# round 5 first call: copy-engine probe (default env and SDMA knobs) and the
# config-3 bench under a kernel trace with the default-stream fix
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
cd /tmp
step probe_default 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/probe_default -o p -- python3 $R/tools/copy_probe.py
HSA_ENABLE_SDMA=1 step probe_sdma1 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/probe_sdma1 -o p -- python3 $R/tools/copy_probe.py
GPU_BLIT_ENGINE_TYPE=2 step probe_blit2 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/probe_blit2 -o p -- python3 $R/tools/copy_probe.py
step genome 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/genome -o g -- python3 -u $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline
exit 0
