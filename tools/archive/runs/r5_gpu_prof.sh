#!/bin/bash
# round-5 close: profile rounds r5v1 (M1) and r5v1m2 (M2) -- large per-dispatch CSVs deleted on the
# box once summarised (the merge-back limit is 64 MiB) -- then the other BASELINE configs
set -o pipefail
mkdir -p gpurun_out
trim() { find gpurun_out/prof_$1 -name '*.csv' ! -name '*kernel_stats.csv' -size +1M -delete; }
timeout -k 10 500 bash tools/profile_round.sh r5v1 > gpurun_out/prof_r5v1.log 2>&1 || { echo "PROFILE M1 FAILED"; tail -20 gpurun_out/prof_r5v1.log; exit 3; }
trim r5v1; tail -1 gpurun_out/prof_r5v1.log
timeout -k 10 380 bash tools/profile_round.sh r5v1m2 --frames84 > gpurun_out/prof_r5v1m2.log 2>&1 || { echo "PROFILE M2 FAILED"; tail -20 gpurun_out/prof_r5v1m2.log; exit 4; }
trim r5v1m2; tail -1 gpurun_out/prof_r5v1m2.log
du -sh gpurun_out
timeout -k 10 900 bash tools/configs_bench.sh
