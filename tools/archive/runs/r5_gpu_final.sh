#!/bin/bash
# round-5 close: the full GPU suite, smoke(), profile rounds r5v1 (M1) and r5v1m2 (M2)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r5_final_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 gpurun_out/r5_final_tests.log; exit 1; }
tail -1 gpurun_out/r5_final_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_final_smoke.log 2>&1 || { tail -20 gpurun_out/r5_final_smoke.log; exit 2; }
tail -1 gpurun_out/r5_final_smoke.log
timeout -k 10 500 bash tools/profile_round.sh r5v1 > gpurun_out/prof_r5v1.log 2>&1 || { echo "PROFILE M1 FAILED"; tail -20 gpurun_out/prof_r5v1.log; exit 3; }
tail -1 gpurun_out/prof_r5v1.log
timeout -k 10 380 bash tools/profile_round.sh r5v1m2 --frames84 > gpurun_out/prof_r5v1m2.log 2>&1 || { echo "PROFILE M2 FAILED"; tail -20 gpurun_out/prof_r5v1m2.log; exit 4; }
tail -1 gpurun_out/prof_r5v1m2.log
