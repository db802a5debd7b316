# diagnostic: request tests on a library whose request_eval_kernel also
# computes the per-chain sums by end captures and prints any disagreement
# with the shipping sums (the shipping sums drive every address)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-endcap}
mkdir -p $OUT
export SBEACON_LIB=$R/tools/endcap_lib/libsbeacon_hip.so
timeout -k 10 400 python3 -u -m pytest $R/tests -m gpu -x -v -s --timeout 120 --timeout-method thread -k "requests or genome or persist or chains or beacon" > $OUT/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -c "^endcap" $OUT/tests.log; grep "^endcap" $OUT/tests.log | head -5 | cut -c1-300; tail -2 $OUT/tests.log
exit $rc
