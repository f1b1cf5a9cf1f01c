#!/bin/bash
# round 5: upper bound of an in-kernel fc -- the rollout with the partial fc skipped (marker build,
# measurement only: results are not valid training) against the same build with it
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
O=gpurun_out/r5g7; mkdir -p $O
MK=async-rl-tensorflow_amd/lib/var/mk/liba3c_hip.so
for rep in 1 2 3; do
  for cfg in "A3C_LIB=$MK" "A3C_LIB=$MK A3C_ABL_FC=1" "A3C_LIB=$MK A3C_ABL_CBWD=1" "A3C_LIB=$MK A3C_ABL_FC=1 A3C_ABL_CBWD=1"; do
    env $cfg timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-kernel-timing --steps 100 --min-seconds 1 > $O/b.json 2>$O/b.err || exit 1
    python3 -c "import json;d=json.load(open('$O/b.json'));print('$cfg'.split('/')[-1], d['value'], d['ms_per_step'])"
  done
done
