#!/bin/bash
# round 5: Q-learning sync bisect over the round-3 commits; C5 kernel trace
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
O=gpurun_out/r5g4; mkdir -p $O
V=async-rl-tensorflow_amd/lib/var
for rep in 1 2; do
  for L in $V/r2/liba3c_hip.so $V/q_600cd3e/liba3c_hip.so $V/q_c34ceed/liba3c_hip.so $V/q_a1633a9/liba3c_hip.so $V/q_a269dc3/liba3c_hip.so $V/q_59abc11/liba3c_hip.so $V/q_94a9663/liba3c_hip.so $V/r3/liba3c_hip.so; do
    A3C_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-kernel-timing --steps 100 --min-seconds 1 --algo q --n-step 32 --update sync > $O/q.json 2>$O/q.err || exit 1
    python3 -c "import json;d=json.load(open('$O/q.json'));print('q-sync', '$L'.split('/')[-2], d['value'])"
  done
done
bash tools/kstats.sh r5c5 --lstm --game SpaceInvaders-v0 || exit 1
