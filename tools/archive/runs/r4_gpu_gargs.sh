#!/bin/bash
# GemmArgs layout restored (maskbits last) against the round-3 build: 1024 envs, C5, M1
set -o pipefail
mkdir -p gpurun_out
V=$PWD/async-rl-tensorflow_amd/lib/var
for args in "--envs 1024" "--lstm --game SpaceInvaders-v0" ""; do
  AB_MODES=overlap AB_REPS=2 AB_ARGS="$args" timeout -k 10 500 bash tools/ab.sh "A3C_X=head" "A3C_LIB=$V/r3/liba3c_hip.so" 2>&1 | grep -v amdgpu.ids | sed "s|$V/||;s|^|[$args] |" || exit 1
done
