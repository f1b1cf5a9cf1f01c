#!/bin/bash
# round 5: one-launch rollout diagnosis -- kernel timings alone and live spans, PERSIST 0 / 1
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
O=gpurun_out/r5g10; mkdir -p $O
for P in 0 1; do
  A3C_PERSIST=$P timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 100 --min-seconds 1 > $O/k$P.json 2>$O/b.err || exit 1
  python3 -c "
import json;d=json.load(open('$O/k$P.json'));k=d.get('kernels',{})
print('PERSIST=$P', d['value'], d['ms_per_step'])
for n,v in k.items(): print('  ', n, {x: v.get(x) for x in ('avg_ms','live_avg_ms','per_iter','live_us_by_step')})"
done
