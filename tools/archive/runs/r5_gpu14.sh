#!/bin/bash
# round 5: M1 re-check of the conv backward's forms on the final build (knobs build, 3 interleaved reps)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
O=gpurun_out/r5g14; mkdir -p $O
K=async-rl-tensorflow_amd/lib/var/knobs/liba3c_hip.so
for rep in 1 2 3; do
  for cfg in "X=0" "A3C_CB_LEAN=1" "A3C_BWD_BOUND=1" "A3C_CB_NWG=224" "A3C_CB_NWG=192"; do
    env A3C_LIB=$K $cfg timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-kernel-timing --steps 100 --min-seconds 1 > $O/b.json 2>$O/b.err || exit 1
    python3 -c "import json;d=json.load(open('$O/b.json'));print('$cfg', d['value'])"
  done
done
