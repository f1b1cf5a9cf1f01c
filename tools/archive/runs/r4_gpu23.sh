#!/bin/bash
# round 4: the phase (c) schedule A/B, then the profile round + SQ counters
set -o pipefail
bash tools/archive/runs/r4_gpu3.sh || exit 1
bash tools/archive/runs/r4_gpu2.sh ${1:-r4v1} || exit 2
