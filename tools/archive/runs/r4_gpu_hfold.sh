#!/bin/bash
# the head weight GEMM's split-K fold in the finalize (default) vs its own k_reduce_slabs, C5 and M1;
# then the LSTM / engine / headline GPU tests on the final wks policy
set -o pipefail
mkdir -p gpurun_out
V=$PWD/async-rl-tensorflow_amd/lib/var
for args in "--lstm --game SpaceInvaders-v0" ""; do
  AB_MODES=overlap AB_REPS=2 AB_ARGS="$args" timeout -k 10 500 bash tools/ab.sh "A3C_X=head" "A3C_HEAD_FOLD=1" "A3C_LIB=$V/r3/liba3c_hip.so" 2>&1 | grep -v amdgpu.ids | sed "s|$V/||;s|^|[$args] |" || exit 1
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_lstm.py tests/test_gpu_engine.py tests/test_gpu_headline_parity.py > gpurun_out/hfold_tests.log 2>&1 || { tail -30 gpurun_out/hfold_tests.log; exit 2; }
tail -1 gpurun_out/hfold_tests.log
