#!/bin/bash
# round 4: A/B of the in-workgroup split-K fc weight GEMM (A3C_FC_WKS) in M1, M2 and sync mode
set -o pipefail
mkdir -p gpurun_out
for args in "" "--frames84" ; do
  echo "### overlap $args"
  AB_ARGS="$args" AB_MODES=overlap AB_REPS=2 timeout -k 10 500 bash tools/ab.sh "A3C_FC_WKS=1" "A3C_FC_WKS=0" 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_wks.txt || exit 1
done
echo "### sync"
AB_MODES=sync AB_REPS=2 timeout -k 10 500 bash tools/ab.sh "A3C_FC_WKS=1" "A3C_FC_WKS=0" 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_wks.txt || exit 1
