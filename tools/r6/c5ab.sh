#!/bin/bash
# C5 (LSTM head) bench lines: fc split on / off (A3C_FC_SPLIT, release knob), two reps
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/${TAG:-r6c5}; mkdir -p $O
for rep in 1 2; do
for fs in 1 0; do
  A3C_FC_SPLIT=$fs timeout -k 10 300 python3 -u bench.py --lstm --game SpaceInvaders-v0 --steps 20 --warmup 5 \
      --no-cpu-baseline > $O/c5_$fs.json 2>/dev/null || exit $?
  python3 -c "
import json
b=json.loads(open('$O/c5_$fs.json').read().strip().splitlines()[-1])
print('fc_split=$fs', b['value'], b['roofline'].get('kernel'), b['roofline'].get('frac'), b['roofline'].get('avg_us'))" | tee -a $O/ab.txt
done
done
