#!/bin/bash
# bisect the round-4 builds on C5 (LSTM) and 1024 envs: r3, the round-4 csrc commits, HEAD
set -o pipefail
mkdir -p gpurun_out
V=$PWD/async-rl-tensorflow_amd/lib/var
CFGS="A3C_X=head"
for c in r3 0f7a1f4 c2dc87b 40345d1 ffd4b67 c4ca6e7; do CFGS="$CFGS A3C_LIB=$V/$c/liba3c_hip.so"; done
AB_MODES=overlap AB_REPS=2 AB_ARGS="--lstm --game SpaceInvaders-v0" timeout -k 10 700 bash tools/ab.sh $CFGS 2>&1 | grep -v amdgpu.ids | sed "s|$V/||" || exit 1
AB_MODES=overlap AB_REPS=1 AB_ARGS="--envs 1024" timeout -k 10 400 bash tools/ab.sh $CFGS 2>&1 | grep -v amdgpu.ids | sed "s|$V/||;s|^|e1024 |" || exit 1
