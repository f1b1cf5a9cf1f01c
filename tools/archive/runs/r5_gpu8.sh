#!/bin/bash
# round 5: rollout wave priority (s_setprio in the rollout kernels) and fc_part W depth A/B (M1, overlap)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
O=gpurun_out/r5g8; mkdir -p $O
V=async-rl-tensorflow_amd/lib/var
for rep in 1 2 3; do
  for L in knobs cbpr1 cbpr3; do
    A3C_LIB=$V/$L/liba3c_hip.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-kernel-timing --steps 100 --min-seconds 1 > $O/b.json 2>$O/b.err || exit 1
    python3 -c "import json;d=json.load(open('$O/b.json'));print('$L', d['value'], d['ms_per_step'])"
  done
done
for L in cbpr3; do
  A3C_LIB=$V/$L/liba3c_hip.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 100 --min-seconds 1 > $O/k_$L.json 2>$O/b.err || exit 1
  python3 -c "
import json;d=json.load(open('$O/k_$L.json'));k=d.get('kernels',{})
print('$L', d['value'], {n: round(1e3*v['avg_ms'],2) for n,v in k.items()})"
done
