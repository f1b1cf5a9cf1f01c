#!/bin/bash
# round 5: bootstrap head on the backward stream (A3C_BOOT_BWD, knobs build): parity + M1 A/B
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
O=gpurun_out/r5g5; mkdir -p $O
K=async-rl-tensorflow_amd/lib/var/knobs/liba3c_hip.so
A3C_LIB=$K A3C_BOOT_BWD=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_headline_parity.py -x -q \
  --timeout 300 --timeout-method thread -k "overlap and not q_ and not sync" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit $rc; }
for rep in 1 2 3; do
  for cfg in "A3C_BOOT_BWD=0" "A3C_BOOT_BWD=1"; do
    env A3C_LIB=$K $cfg timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 200 --min-seconds 1.5 > $O/ab.json 2>$O/ab.err || exit 1
    python3 -c "import json;d=json.load(open('$O/ab.json'));print('$cfg', d['value'], d['roofline']['avg_us'], d['kernels']['k_head_screen_conv12'].get('live_us_by_step'))"
  done
done
