#!/bin/bash
# round 4: full GPU suite of this build, then the r3-vs-r4 A/B (tools/archive/runs/r4_gpu4.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/r4_gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 gpurun_out/r4_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4_gpu_tests.log
bash tools/archive/runs/r4_gpu4.sh
