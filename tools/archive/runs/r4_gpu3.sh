#!/bin/bash
# round 4: conv backward LDS layouts -- parity of the phase (b) permutation variant, then the A/B of
# the phase (c) schedule (default: bank-spread; cbold: round 3) and of the phase (b) permutation
# (phbperm), M1 and M2, with the kernel alone (AB_KT)
set -o pipefail
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
VO=$R/async-rl-tensorflow_amd/lib/var/cbold/liba3c_hip.so
VP=$R/async-rl-tensorflow_amd/lib/var/phbperm/liba3c_hip.so
A3C_LIB=$VP timeout -k 10 400 python -u -m pytest tests/test_gpu_headline_parity.py tests/test_gpu_engine.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r4_phbperm_tests.log 2>&1 || { echo "PHBPERM TESTS FAILED"; tail -30 gpurun_out/r4_phbperm_tests.log; exit 1; }
tail -2 gpurun_out/r4_phbperm_tests.log
echo "### M1 overlap"
AB_KT=k_conv_bwd AB_MODES=overlap AB_REPS=3 timeout -k 10 600 bash tools/ab.sh "A3C_X=1" "A3C_LIB=$VO" "A3C_LIB=$VP" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_cbsched.txt || exit 1
echo "### M2 overlap"
AB_KT=k_conv_bwd AB_ARGS=--frames84 AB_MODES=overlap AB_REPS=2 timeout -k 10 600 bash tools/ab.sh "A3C_X=1" "A3C_LIB=$VO" "A3C_LIB=$VP" 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_cbsched.txt || exit 1
