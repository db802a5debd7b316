# GPU tests touched this round (region files, pipeline, dedup, summarise, abi)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_summarise.py tests/test_gpu_pipeline.py tests/test_gpu_dedup.py -m gpu -x -v --timeout 300 --timeout-method thread > $R/gpurun_out/gpu_new.log 2>&1; rc=$?
echo "rc=$rc"; tail -15 $R/gpurun_out/gpu_new.log | cut -c1-300
exit $rc
