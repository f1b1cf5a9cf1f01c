#!/bin/bash
# q-learning overlap: the new parity tests, then bench q sync vs overlap (n-step 5 and 32).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_engine.py -k "q_overlap" tests/test_gpu_multirank.py > gpurun_out/qov_tests.log 2>&1 || { tail -40 gpurun_out/qov_tests.log; exit 1; }
tail -3 gpurun_out/qov_tests.log
for u in sync overlap sync overlap; do
  timeout -k 10 120 python -u bench.py --algo q --update $u --steps 200 --warmup 20 --no-cpu-baseline >> gpurun_out/qov_bench.log 2>&1 || exit 1
done
cat gpurun_out/qov_bench.log | grep '"metric"'
