#!/bin/bash
# round 5: fused-kernel phase stamps (MFMA vs VALU screen), then the new feature tests
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
O=gpurun_out/r5g2; mkdir -p $O
for v in hsm hsv; do
  echo "== $v alone"; A3C_LIB=async-rl-tensorflow_amd/lib/var/$v/liba3c_hip.so HS_KER=5 HS_OVERLAP=1 timeout -k 10 120 python3 tools/hs_phases.py 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_lstm.py tests/test_gpu_loopback.py tests/test_gpu_headline_parity.py \
  tests/test_gpu_multirank.py -x -q --timeout 400 --timeout-method thread \
  -k "lstm or loopback or c4 or c5 or hogwild or split_exchange" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit $rc; }
exit 0
