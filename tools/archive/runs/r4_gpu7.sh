#!/bin/bash
# round 4: parity of this build's backward (headline + engine tests), the wks GEMM's XCD order A/B,
# and the M1 knob re-sweep
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_headline_parity.py tests/test_gpu_engine.py tests/test_gpu_multirank.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r4_quick_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/r4_quick_tests.log; exit 1; }
tail -2 gpurun_out/r4_quick_tests.log
AB_MODES=overlap AB_REPS=2 timeout -k 10 400 bash tools/ab.sh "A3C_X=1" "A3C_WKS_XCD=0" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_wksxcd.txt || exit 1
bash tools/archive/runs/r4_gpu6.sh
# the fused rollout kernel's phase timestamps alone (one workgroup, -DHS_TIMES build)
R=${GRAFT_REPO_ROOT:-$(pwd)}
A3C_LIB=$R/async-rl-tensorflow_amd/lib/var/hstimes/liba3c_hip.so HS_KER=5 HS_OVERLAP=1 timeout -k 10 120 python3 tools/hs_phases.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/hs_phases_r4.txt
# the conv backward's per-phase time alone (-DCB_PHASES build)
A3C_LIB=$R/async-rl-tensorflow_amd/lib/var/cbp/liba3c_hip.so timeout -k 10 120 python3 tools/cb_phases.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/cb_phases_r4.txt
