#!/bin/bash
# which round-4 change costs C5 (LSTM) and 1024 envs: the in-workgroup split-K fc weight GEMM
# (A3C_FC_WKS) or the ReLU bits (A3C_L2BITS), interleaved
set -o pipefail
mkdir -p gpurun_out
for args in "--lstm --game SpaceInvaders-v0" "--envs 1024"; do
  AB_MODES=overlap AB_REPS=2 AB_ARGS="$args" timeout -k 10 700 bash tools/ab.sh "A3C_X=r4" "A3C_FC_WKS=0" "A3C_L2BITS=0" 2>&1 | grep -v amdgpu.ids | sed "s|^|[$args] |" || exit 1
done
