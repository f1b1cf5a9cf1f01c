#!/bin/bash
# round 5: config A/Bs vs the round-4-design build (r5a), and Q-learning sync across round builds
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
O=gpurun_out/r5g2b; mkdir -p $O
OLD=async-rl-tensorflow_amd/lib/var/r5a/liba3c_hip.so
for cfg in "--lstm --game SpaceInvaders-v0" "--envs 512 --update hogwild" "--envs 512" "--envs 512 --update hogwild --hogwild-sync"; do
  for rep in 1 2; do
    for L in "" "$OLD"; do
      [ -n "$L" ] && [ "$cfg" = "--envs 512 --update hogwild" ] && continue   # (r5a has no overlapped hogwild)
      A3C_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-kernel-timing --steps 200 --min-seconds 1 $cfg > $O/ab.json 2>$O/ab.err || exit 1
      python3 -c "import json;d=json.load(open('$O/ab.json'));print('$cfg', '${L:-new}', d['value'])"
    done
  done
done
for rep in 1 2; do
  for L in "" async-rl-tensorflow_amd/lib/var/r2/liba3c_hip.so async-rl-tensorflow_amd/lib/var/r3/liba3c_hip.so async-rl-tensorflow_amd/lib/var/r4/liba3c_hip.so; do
    A3C_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-kernel-timing --steps 100 --min-seconds 1 --algo q --n-step 32 --update sync > $O/q.json 2>$O/q.err || exit 1
    python3 -c "import json;d=json.load(open('$O/q.json'));print('q-sync', '${L:-new}', d['value'])"
  done
done
