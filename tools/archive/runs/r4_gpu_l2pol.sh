#!/bin/bash
# the ReLU-bit policy (bits where the backward bounds, ballot compiled out elsewhere) against
# forced bits and the round-3 build; then the engine / checkpoint / headline GPU tests
set -o pipefail
mkdir -p gpurun_out
V=$PWD/async-rl-tensorflow_amd/lib/var
for args in "" "--frames84" "--lstm --game SpaceInvaders-v0" "--envs 1024"; do
  AB_MODES=overlap AB_REPS=2 AB_ARGS="$args" timeout -k 10 600 bash tools/ab.sh "A3C_X=policy" "A3C_L2BITS=1" "A3C_LIB=$V/r3/liba3c_hip.so" 2>&1 | grep -v amdgpu.ids | sed "s|$V/||;s|^|[$args] |" || exit 1
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_engine.py tests/test_gpu_checkpoint.py tests/test_gpu_headline_parity.py tests/test_gpu_lstm.py > gpurun_out/l2pol_tests.log 2>&1 || { tail -30 gpurun_out/l2pol_tests.log; exit 2; }
tail -2 gpurun_out/l2pol_tests.log
