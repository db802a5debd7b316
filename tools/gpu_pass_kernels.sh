# request pass: the request GPU tests, the rotating-batch digest / timing,
# and every kernel's duration from a kernel trace (tools/kernel_table.py)
mkdir -p gpurun_out/${TAG:-gpu_pass_kernels}
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-gpu_pass_kernels}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-400
  case $rc in 0) return 0;; *) exit $rc;; esac
}
step tests 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_requests.py tests/test_gpu_persist.py
step full 300 python3 -u $R/tools/req_tune.py --save /tmp/st --digest
cd /tmp
step prof 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o t -- python3 -u $R/tools/req_tune.py --open /tmp/st --rounds 5
python3 $R/tools/kernel_table.py $O/prof/t_kernel_trace.csv 12 > $O/kernels.txt; cat $O/kernels.txt | cut -c1-140
exit 0
