#!/bin/bash
# round-4 close, final build: the full GPU suite, smoke(), profile rounds r4v4 (M1) and r4v4m2 (M2)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r4_final_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 gpurun_out/r4_final_tests.log; exit 1; }
tail -1 gpurun_out/r4_final_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_final_smoke.log 2>&1 || { tail -20 gpurun_out/r4_final_smoke.log; exit 2; }
tail -1 gpurun_out/r4_final_smoke.log
timeout -k 10 500 bash tools/profile_round.sh r4v4 > gpurun_out/prof_r4v4.log 2>&1 || { echo "PROFILE M1 FAILED"; tail -20 gpurun_out/prof_r4v4.log; exit 3; }
tail -1 gpurun_out/prof_r4v4.log
timeout -k 10 380 bash tools/profile_round.sh r4v4m2 --frames84 > gpurun_out/prof_r4v4m2.log 2>&1 || { echo "PROFILE M2 FAILED"; tail -20 gpurun_out/prof_r4v4m2.log; exit 4; }
tail -1 gpurun_out/prof_r4v4m2.log
