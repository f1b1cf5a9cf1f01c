#!/bin/bash
# C5 kernel stats (rocprofv3 --kernel-trace --stats) with the fc fold in either place
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6c5p}; mkdir -p $O
for ff in ${FOLDS:-0 1}; do
  A3C_LSTM_FCFOLD=$ff timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p$ff -o run --output-format csv -- \
      python3 -u bench.py --lstm --game SpaceInvaders-v0 --steps 20 --warmup 5 --no-cpu-baseline > $O/b$ff.json 2>$O/err$ff.log || exit $?
  f=$(find $O/p$ff -name '*kernel_stats.csv' | head -1)
  cp "$f" $O/kstats_fold$ff.csv && rm -rf $O/p$ff || exit 1
done
