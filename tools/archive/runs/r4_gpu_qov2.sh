#!/bin/bash
# q-learning overlap on partitioned-PS ranks (gloo on one GPU) against the oracle.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_multirank.py -k "q" > gpurun_out/qov2_tests.log 2>&1 || { tail -60 gpurun_out/qov2_tests.log; exit 1; }
tail -15 gpurun_out/qov2_tests.log
# rollout-stream kernel gaps: a plain kernel trace of a short M1 bench (tools/kgaps.py reads it)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ktrace -o kt -- \
  python3 bench.py --steps 60 --warmup 20 --no-cpu-baseline > gpurun_out/ktrace_bench.log 2>&1 || { tail -20 gpurun_out/ktrace_bench.log; exit 1; }
find gpurun_out/ktrace -name '*.csv'
