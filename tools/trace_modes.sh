#!/bin/bash
# Kernel traces (with timestamps) of the default bench in overlap and sync mode, for tools/timeline.py.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-tl}; shift
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
for mode in overlap sync; do
  O=gpurun_out/$TAG/$mode; mkdir -p $O
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
    python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-kernel-timing --min-seconds 0 --update $mode "$@" \
    > $O/bench.json 2> $O/err.log || exit 1
  f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
  python3 tools/timeline.py "$f" k_prep_fwd 40 > $O/timeline.txt || exit 1
  cp "$f" $O/kernel_trace.csv
  cat $O/timeline.txt
done
