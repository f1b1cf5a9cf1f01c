#!/bin/bash
# round 4: this build against the round-3 build (lib/var/r3, the same sources as commit 45d25c1)
# and its knobs: the in-workgroup split-K fc weight GEMM (A3C_FC_WKS), the dl2 ReLU bits (A3C_L2BITS)
set -o pipefail
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
V3=$R/async-rl-tensorflow_amd/lib/var/r3/liba3c_hip.so
echo "### M1 overlap"
AB_MODES=overlap AB_REPS=2 timeout -k 10 500 bash tools/ab.sh "A3C_X=1" "A3C_LIB=$V3" "A3C_FC_WKS=0" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_r3.txt || exit 1
echo "### M2 overlap"
AB_ARGS=--frames84 AB_MODES=overlap AB_REPS=2 timeout -k 10 500 bash tools/ab.sh "A3C_X=1" "A3C_LIB=$V3" "A3C_L2BITS=0" 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_r3.txt || exit 1
echo "### sync"
AB_MODES=sync AB_REPS=2 timeout -k 10 400 bash tools/ab.sh "A3C_X=1" "A3C_LIB=$V3" 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_r3.txt || exit 1
