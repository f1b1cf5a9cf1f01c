#!/bin/bash
# A/B of engine knobs: tools/ab.sh "ENV=1" "ENV=2" ... ; each config x 3 reps x {sync,overlap}, interleaved
for rep in 1 2 3; do
  for cfg in "$@"; do
    for u in sync overlap; do
      env $cfg timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-kernel-timing --steps 400 --update $u > gpurun_out/ab.json || exit 1
      python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$cfg', '$u', d['value'])"
    done
  done
done
