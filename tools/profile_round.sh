#!/bin/bash
# One profiling round on the GPU box:  tools/profile_round.sh TAG [bench args...]
# bench line, rocprofv3 kernel-trace/stats, two PMC passes (FETCH_SIZE, WRITE_SIZE), summary.
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
echo "[profile] bench" && \
timeout -k 10 400 python3 bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" && cat "$OUT/bench.json" && \
echo "[profile] kernel trace" && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 100 --no-cpu-baseline "$@" > "$OUT/trace.log" 2>&1 && \
echo "[profile] pmc FETCH_SIZE" && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing "$@" > "$OUT/pmc_fetch.log" 2>&1 && \
echo "[profile] pmc WRITE_SIZE" && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing "$@" > "$OUT/pmc_write.log" 2>&1 && \
python3 tools/pmc_summarize.py "$OUT" > "$OUT/summary.json" && echo "[profile] done"
