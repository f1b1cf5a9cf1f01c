#!/bin/bash
# C5 / 1024-env regression: the forward ballot compiled out (nol2m), the GEMM MASKBITS epilogue
# compiled out (nomb), against the default build and round 3; all with A3C_L2BITS=0 (l2 re-read)
set -o pipefail
mkdir -p gpurun_out
V=$PWD/async-rl-tensorflow_amd/lib/var
for args in "--lstm --game SpaceInvaders-v0" "--envs 1024"; do
  AB_MODES=overlap AB_REPS=2 AB_ARGS="$args" timeout -k 10 600 bash tools/ab.sh "A3C_L2BITS=0" "A3C_L2BITS=0 A3C_LIB=$V/nol2m/liba3c_hip.so" "A3C_L2BITS=0 A3C_LIB=$V/nomb/liba3c_hip.so" "A3C_LIB=$V/r3/liba3c_hip.so" 2>&1 | grep -v amdgpu.ids | sed "s|$V/||;s|^|[$args] |" || exit 1
done
