#!/bin/bash
# isolate a nature parity failure: the sync parity case under knob settings (knobs build)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/${TAG:-r6iso}; mkdir -p $O
V=$ROOT/async-rl-tensorflow_amd/lib/var/knobs
make -C async-rl-tensorflow_amd/csrc -s -j16 OUT=$V/liba3c_hip.so OBJDIR=$V/obj EXTRA=-DA3C_KNOBS > $O/build.log 2>&1 || exit $?
IFS=';' read -ra LIST <<< "${CFGS:-A3C_NAT_FUSE_DX=0}"
for cfg in "${LIST[@]}"; do
  env A3C_LIB=$V/liba3c_hip.so $cfg timeout -k 10 200 python3 -u -m pytest tests/test_gpu_nature.py -x -q --timeout 150 \
      --timeout-method thread -k "sync_matches_oracle and 6-8" > $O/t.log 2>&1
  rc=$?
  echo "$cfg rc=$rc $(grep -o "AssertionError.*" $O/t.log | head -1)" | tee -a $O/iso.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
