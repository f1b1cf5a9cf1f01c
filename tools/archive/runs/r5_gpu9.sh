#!/bin/bash
# round 5: the one-launch rollout (k_rollout_persist) -- bit-exactness vs the multi-launch form,
# engine parity, then the M1 bench A/B (A3C_PERSIST=0 / 1)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
O=gpurun_out/r5g9; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_persist.py > $O/persist.log 2>&1 || { tail -40 $O/persist.log; exit 1; }
tail -3 $O/persist.log
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py tests/test_gpu_headline_parity.py > $O/eng.log 2>&1 || { tail -40 $O/eng.log; exit 1; }
tail -2 $O/eng.log
for rep in 1 2 3; do
  for P in 0 1; do
    A3C_PERSIST=$P timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-kernel-timing --steps 100 --min-seconds 1 > $O/b.json 2>$O/b.err || exit 1
    python3 -c "import json;d=json.load(open('$O/b.json'));print('PERSIST=$P', d['value'], d['ms_per_step'])"
  done
done
