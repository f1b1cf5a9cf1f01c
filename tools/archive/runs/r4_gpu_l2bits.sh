#!/bin/bash
# the ReLU bits end to end: A3C_L2BITS=0 now also drops the forward's ballot (M1, M2, C5, 1024 envs)
set -o pipefail
mkdir -p gpurun_out
for args in "" "--frames84" "--lstm --game SpaceInvaders-v0" "--envs 1024"; do
  AB_MODES=overlap AB_REPS=2 AB_ARGS="$args" timeout -k 10 500 bash tools/ab.sh "A3C_L2BITS=1" "A3C_L2BITS=0" 2>&1 | grep -v amdgpu.ids | sed "s|^|[$args] |" || exit 1
done
