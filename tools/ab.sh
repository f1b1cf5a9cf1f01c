#!/bin/bash
# A/B of engine knobs: tools/ab.sh "ENV=1" "ENV=2" ... ; each config x AB_REPS reps x AB_MODES, interleaved.
# AB_KT=k_name: also time that kernel (bench.py kernel timing) and print its average.
# AB_MODES (default "sync overlap"), AB_REPS (default 3), AB_ARGS: extra bench.py arguments.
KT=${AB_KT:-}
MODES=${AB_MODES:-sync overlap}
REPS=${AB_REPS:-3}
for rep in $(seq 1 "$REPS"); do
  for cfg in "$@"; do
    for u in $MODES; do
      if [ -n "$KT" ]; then kt=""; else kt="--no-kernel-timing"; fi
      env $cfg timeout -k 10 200 python3 bench.py --no-cpu-baseline $kt --steps 400 --update $u $AB_ARGS > gpurun_out/ab.json || exit 1
      python3 -c "
import json;d=json.load(open('gpurun_out/ab.json'))
k='$KT'
print('$cfg', '$u', d['value'], (k + ' %.1f us' % (1e3 * d['kernels'][k]['avg_ms'])) if k else '')"
    done
  done
done
