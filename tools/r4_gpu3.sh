#!/bin/bash
# round 4: A/B of the conv backward's phase (c) schedule (bank-spread vs round 3), M1 and M2, plus
# the kernel alone (AB_KT)
set -o pipefail
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/async-rl-tensorflow_amd/lib/var/cbold/liba3c_hip.so
[ -f "$V" ] || V=$(pwd)/async-rl-tensorflow_amd/lib/var/cbold/liba3c_hip.so
echo "### M1 overlap"
AB_KT=k_conv_bwd AB_MODES=overlap AB_REPS=3 timeout -k 10 600 bash tools/ab.sh "A3C_X=1" "A3C_LIB=$V" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_cbsched.txt || exit 1
echo "### M2 overlap"
AB_KT=k_conv_bwd AB_ARGS=--frames84 AB_MODES=overlap AB_REPS=3 timeout -k 10 600 bash tools/ab.sh "A3C_X=1" "A3C_LIB=$V" 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_cbsched.txt || exit 1
