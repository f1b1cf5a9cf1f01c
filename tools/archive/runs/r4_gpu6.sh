#!/bin/bash
# round 4: knob re-sweep of the M1 overlap schedule on this build
set -o pipefail
mkdir -p gpurun_out
AB_MODES=overlap AB_REPS=2 timeout -k 10 1000 bash tools/ab.sh "A3C_X=1" "A3C_CB_NWG=224" "A3C_CB_NWG=192" \
  "A3C_FCP_KS=2" "A3C_ROLLOUT_PRIO=0" "A3C_GEMM_XCD=1" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_knobs.txt || exit 1
