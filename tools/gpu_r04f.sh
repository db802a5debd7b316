#!/bin/bash
# persisted stores on the device: tests, then the config-3 save/open timing
set -o pipefail
mkdir -p gpurun_out/r04f
df -h /tmp . > gpurun_out/r04f/df.txt 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_persist.py \
  > gpurun_out/r04f/pytest.log 2>&1 &&
timeout -k 10 600 python -u tools/persist_bench.py > gpurun_out/r04f/persist.json 2> gpurun_out/r04f/persist.err
