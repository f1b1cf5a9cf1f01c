#!/bin/bash
# round 5: C5 (LSTM head, SpaceInvaders, 256 envs) -- the backward-bound choices, partial-fc K split, GEMM forms
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
O=gpurun_out/r5g12; mkdir -p $O
K=async-rl-tensorflow_amd/lib/var/knobs/liba3c_hip.so
for rep in 1 2 3; do
  for cfg in "X=0" "A3C_BWD_BOUND=1" "A3C_FCP_KS=2" "A3C_GEMM_MULTI=1" "A3C_LATE_GO=0" "A3C_HEAD_FOLD=0"; do
    env A3C_LIB=$K $cfg timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-kernel-timing --steps 100 --min-seconds 1 --lstm --game SpaceInvaders-v0 > $O/b.json 2>$O/b.err || exit 1
    python3 -c "import json;d=json.load(open('$O/b.json'));print('$cfg', d['value'])"
  done
done
