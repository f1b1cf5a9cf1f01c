#!/bin/bash
# C5 (LSTM head): the fc fold in the cell kernel (A3C_LSTM_FCFOLD=0) or once per fc tile in the
# fc launch (k_fc_part_fold, =1); whole-bench lines, alternating, three reps
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/${TAG:-r6c5f}; mkdir -p $O
for rep in 1 2 3; do
for ff in 0 1; do
  A3C_LSTM_FCFOLD=$ff timeout -k 10 300 python3 -u bench.py --lstm --game SpaceInvaders-v0 --steps 20 --warmup 5 \
      --no-cpu-baseline > $O/c5_$ff.json 2>/dev/null || exit $?
  python3 -c "
import json
b=json.loads(open('$O/c5_$ff.json').read().strip().splitlines()[-1])
print('fcfold=$ff', b['value'], b['roofline'].get('kernel'), b['roofline'].get('frac'), b['roofline'].get('avg_us'))" | tee -a $O/ab.txt
done
done
