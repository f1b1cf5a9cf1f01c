#!/bin/bash
# buffer placement: the ReLU-bit buffers allocated last (default build) vs between act_l2 and act_l3
# (var/cur) vs the round-3 build, on C5 (LSTM), 1024 envs and M1
set -o pipefail
mkdir -p gpurun_out
V=$PWD/async-rl-tensorflow_amd/lib/var
for args in "--lstm --game SpaceInvaders-v0" "--envs 1024" ""; do
  AB_MODES=overlap AB_REPS=2 AB_ARGS="$args" timeout -k 10 500 bash tools/ab.sh "A3C_X=last" "A3C_LIB=$V/cur/liba3c_hip.so" "A3C_LIB=$V/r3/liba3c_hip.so" 2>&1 | grep -v amdgpu.ids | sed "s|$V/||;s|^|[$args] |" || exit 1
done
