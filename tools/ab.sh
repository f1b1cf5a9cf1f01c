#!/bin/bash
# A/B of engine knobs: tools/ab.sh "ENV=1" "ENV=2" ... ; each config x 3 reps x {sync,overlap}, interleaved.
# AB_KT=k_name: also time that kernel (bench.py kernel timing) and print its average.
KT=${AB_KT:-}
for rep in 1 2 3; do
  for cfg in "$@"; do
    for u in sync overlap; do
      if [ -n "$KT" ]; then kt=""; else kt="--no-kernel-timing"; fi
      env $cfg timeout -k 10 200 python3 bench.py --no-cpu-baseline $kt --steps 400 --update $u > gpurun_out/ab.json || exit 1
      python3 -c "
import json;d=json.load(open('gpurun_out/ab.json'))
k='$KT'
print('$cfg', '$u', d['value'], (k + ' %.1f us' % (1e3 * d['kernels'][k]['avg_ms'])) if k else '')"
    done
  done
done
