#!/bin/bash
# round 5: one-launch rollout ablations (measurement only): no fc tiles / no hand-off waits / both;
# pkp = kernel arguments read per step through the kernarg pointer
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
O=gpurun_out/r5g11; mkdir -p $O
V=async-rl-tensorflow_amd/lib/var
for L in knobs pv_nosleep pv_onlya pv_plainst; do
  A3C_LIB=$V/$L/liba3c_hip.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 100 --min-seconds 1 > $O/k.json 2>$O/b.err || exit 1
  python3 -c "
import json;d=json.load(open('$O/k.json'));k=d.get('kernels',{})
r=k.get('k_rollout_persist',{}); h=k.get('k_head_screen_conv12',{})
print('$L', d['value'], 'persist alone', r.get('avg_ms'), 'live', r.get('live_avg_ms'), 'steps live', h.get('live_us_by_step'), 'cbwd live', k.get('k_conv_bwd',{}).get('live_avg_ms'))"
done
