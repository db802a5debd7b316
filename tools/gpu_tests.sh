mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -30 gpurun_out/gpu_tests.log; exit $rc
