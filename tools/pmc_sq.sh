#!/bin/bash
# SQ counter pass (one rocprofv3 --pmc run, 8 SQ counters) of a short bench: tools/pmc_sq.sh TAG [bench args]
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/sq_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
A3C_WAIT_VALUE=0 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d "$OUT/pmc" -o run --output-format csv -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing "$@" > "$OUT/pmc.log" 2>&1 && \
python3 tools/pmc_kernels.py "$OUT/pmc" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
