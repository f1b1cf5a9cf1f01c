#!/bin/bash
# round 5, call 2: LSTM fold, loopback exchange, hogwild overlap tests; config A/Bs vs the r5a build
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
O=gpurun_out/r5g2; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_lstm.py tests/test_gpu_loopback.py tests/test_gpu_headline_parity.py \
  tests/test_gpu_multirank.py -x -q --timeout 400 --timeout-method thread \
  -k "lstm or loopback or c4 or c5 or hogwild or split_exchange" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit $rc; }
OLD=async-rl-tensorflow_amd/lib/var/r5a/liba3c_hip.so
for cfg in "--lstm --game SpaceInvaders-v0" "--envs 512 --update hogwild" "--envs 512"; do
  for rep in 1 2; do
    for L in "" "$OLD"; do
      A3C_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-kernel-timing --steps 200 $cfg > $O/ab.json 2>$O/ab.err || exit 1
      python3 -c "import json;d=json.load(open('$O/ab.json'));print('$cfg', '${L:-new}', d['value'])"
    done
  done
done
# Q-learning sync across the round builds (3.48M round 2 -> 3.41M rounds 3-4)
for rep in 1 2; do
  for L in "" async-rl-tensorflow_amd/lib/var/r2/liba3c_hip.so async-rl-tensorflow_amd/lib/var/r3/liba3c_hip.so async-rl-tensorflow_amd/lib/var/r4/liba3c_hip.so; do
    A3C_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-kernel-timing --steps 100 --algo q --n-step 32 --update sync > $O/q.json 2>$O/q.err || exit 1
    python3 -c "import json;d=json.load(open('$O/q.json'));print('q-sync', '${L:-new}', d['value'])"
  done
done
