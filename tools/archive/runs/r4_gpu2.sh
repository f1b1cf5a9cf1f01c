#!/bin/bash
# round 4: profile round of the default bench (kernel trace + HBM PMC passes) and one SQ counter pass
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r4v1}
timeout -k 10 900 bash tools/profile_round.sh $TAG > gpurun_out/prof_$TAG.log 2>&1 || { echo "PROFILE FAILED"; tail -30 gpurun_out/prof_$TAG.log; exit 1; }
tail -3 gpurun_out/prof_$TAG.log
timeout -k 10 200 bash tools/pmc_sq.sh $TAG > gpurun_out/sq_$TAG.log 2>&1 || { echo "SQ FAILED"; tail -20 gpurun_out/sq_$TAG.log; exit 2; }
cat gpurun_out/sq_$TAG.log | head -30
