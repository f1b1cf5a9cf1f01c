#!/bin/bash
# SQ counter passes over a bench run: tools/pmc_round.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
# counter collection serialises dispatches across queues: the overlap pipeline's wait-value stream
# ordering would wait on a dispatch held behind it (the run hangs), so the passes use event ordering
export A3C_WAIT_VALUE=0
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_WAVES"
timeout -k 10 300 rocprofv3 --pmc $P1 -d "$OUT/p1" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing "$@" > "$OUT/p1.log" 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc $P2 -d "$OUT/p2" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing "$@" > "$OUT/p2.log" 2>&1 && \
python3 tools/pmc_kernels.py "$OUT/p1" "$OUT/p2" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
