# FETCH_SIZE calibration: known-byte reads at 4 / 8 / 16 B per lane and a
# random 64-B-line gather, one --pmc FETCH_SIZE pass (kernel trace only)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_calib -o run -- $R/tools/bin/fetch_calib > $R/gpurun_out/pmc_calib.log 2>&1
rc=$?; echo "calib rc=$rc"; grep '^{' $R/gpurun_out/pmc_calib.log
exit $rc
