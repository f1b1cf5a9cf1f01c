#!/bin/bash
# round 5: C5 -- k_lstm_fwd capped at 128 VGPRs (co-resides with the conv backward) and its load order
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
O=gpurun_out/r5g15; mkdir -p $O
V=async-rl-tensorflow_amd/lib/var
for rep in 1 2 3 4 5; do
  for L in lstm_head lstm_reord lstm_w4; do
    A3C_LIB=$V/$L/liba3c_hip.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-kernel-timing --steps 100 --min-seconds 1 --lstm --game SpaceInvaders-v0 > $O/b.json 2>$O/b.err || exit 1
    python3 -c "import json;d=json.load(open('$O/b.json'));print('$L', d['value'])"
  done
done
