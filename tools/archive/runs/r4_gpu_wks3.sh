#!/bin/bash
# the fc weight GEMM's in-workgroup split-K up to B = 1280 (default) vs up to 2560 at 512 envs (C4),
# and C5 (LSTM) with it off
set -o pipefail
mkdir -p gpurun_out
V=$PWD/async-rl-tensorflow_amd/lib/var
AB_MODES=overlap AB_REPS=2 AB_ARGS="--envs 512" timeout -k 10 500 bash tools/ab.sh "A3C_X=head" "A3C_FC_WKS_MAXB=2560" "A3C_LIB=$V/r3/liba3c_hip.so" 2>&1 | grep -v amdgpu.ids | sed "s|$V/||;s|^|[512] |" || exit 1
AB_MODES=overlap AB_REPS=2 AB_ARGS="--lstm --game SpaceInvaders-v0" timeout -k 10 500 bash tools/ab.sh "A3C_X=head" "A3C_FC_WKS=0" 2>&1 | grep -v amdgpu.ids | sed "s|^|[lstm] |" || exit 1
