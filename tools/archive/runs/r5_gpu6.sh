#!/bin/bash
# round 5: epsilon schedule inside the head kernel -- Q parity tests, then Q-sync A/B vs HEAD~
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
O=gpurun_out/r5g6; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_engine.py tests/test_gpu_dropin.py tests/test_gpu_checkpoint.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
V=async-rl-tensorflow_amd/lib/var
for rep in 1 2 3; do
  for L in $V/q_head/liba3c_hip.so async-rl-tensorflow_amd/lib/liba3c_hip.so; do
    A3C_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-kernel-timing --steps 100 --min-seconds 1 --algo q --n-step 32 --update sync > $O/q.json 2>$O/q.err || exit 1
    python3 -c "import json;d=json.load(open('$O/q.json'));print('q-sync', '$L'.split('/')[-2], d['value'])"
  done
done
