#!/bin/bash
# round 4 final configuration: profile rounds of M1 (r4v2) and M2 (r4v2m2) -- kernel trace, HBM PMC
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 bash tools/profile_round.sh r4v2 > gpurun_out/prof_r4v2.log 2>&1 || { echo "PROFILE M1 FAILED"; tail -20 gpurun_out/prof_r4v2.log; exit 1; }
tail -2 gpurun_out/prof_r4v2.log
timeout -k 10 380 bash tools/profile_round.sh r4v2m2 --frames84 > gpurun_out/prof_r4v2m2.log 2>&1 || { echo "PROFILE M2 FAILED"; tail -20 gpurun_out/prof_r4v2m2.log; exit 2; }
tail -2 gpurun_out/prof_r4v2m2.log
