#!/bin/bash
# LDS / VALU counter pass per kernel (what the co-resident rollout is sensitive to; tools/probe12.sh)
#   tools/pmc_lds.sh TAG [bench args]
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/lds_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
A3C_WAIT_VALUE=0 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT \
  SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS -d "$OUT/pmc" -o run --output-format csv -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing "$@" > "$OUT/pmc.log" 2>&1 && \
python3 tools/pmc_kernels.py "$OUT/pmc" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
