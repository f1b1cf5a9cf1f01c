#!/bin/bash
# The two PMC passes + summary of an existing profiling round (tools/profile_round.sh TAG ran the
# bench and the kernel trace): tools/pmc_only.sh TAG
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
echo "[profile] pmc FETCH_SIZE" && \
A3C_WAIT_VALUE=0 timeout -k 10 150 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing "$@" > "$OUT/pmc_fetch.log" 2>&1 && \
echo "[profile] pmc WRITE_SIZE" && \
A3C_WAIT_VALUE=0 timeout -k 10 150 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing "$@" > "$OUT/pmc_write.log" 2>&1 && \
python3 tools/pmc_summarize.py "$OUT" > "$OUT/summary.json" && echo "[profile] done"
