#!/bin/bash
# quick GPU check: engine tests, sync+overlap bench, sync kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_kernels.py tests/test_gpu_lstm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1; echo rc=$? >> gpurun_out/ab_tests.log
timeout -k 10 200 python3 bench.py --no-cpu-baseline --update sync > gpurun_out/ab_sync.json 2>/dev/null
timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/ab_ov.json 2>/dev/null
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_trace -o run --output-format csv -- python3 bench.py --steps 60 --update sync --no-cpu-baseline --no-kernel-timing > gpurun_out/ab_trace.log 2>&1
