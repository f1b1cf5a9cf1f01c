#!/bin/bash
# round 4: profile round of the default bench (kernel trace + HBM PMC passes), then the A/B of
# the dl2 epilogue's ReLU bits (A3C_L2BITS) in the headline overlap mode
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r4v1}
timeout -k 10 900 bash tools/profile_round.sh $TAG > gpurun_out/prof_$TAG.log 2>&1 || { echo "PROFILE FAILED"; tail -30 gpurun_out/prof_$TAG.log; exit 1; }
tail -3 gpurun_out/prof_$TAG.log
AB_MODES=overlap AB_REPS=3 timeout -k 10 600 bash tools/ab.sh "A3C_L2BITS=1" "A3C_L2BITS=0" 2>&1 | tee gpurun_out/ab_l2bits.txt
