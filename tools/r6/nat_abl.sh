#!/bin/bash
# nature passes: release vs no-MFMA (NAT_ABL=1) vs no-operand-loads (NAT_ABL=2) builds
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/${TAG:-r6abl}; mkdir -p $O
for v in 1 2; do
  V=$ROOT/async-rl-tensorflow_amd/lib/var/abl$v
  make -C async-rl-tensorflow_amd/csrc -s -j16 OUT=$V/liba3c_hip.so OBJDIR=$V/obj EXTRA=-DNAT_ABL=$v > $O/build$v.log 2>&1 || exit $?
done
timeout -k 10 120 python3 -u tools/r6/nat_abl.py > $O/rel.json || exit $?
for v in 1 2; do
  A3C_LIB=$ROOT/async-rl-tensorflow_amd/lib/var/abl$v/liba3c_hip.so timeout -k 10 120 python3 -u tools/r6/nat_abl.py > $O/abl$v.json || exit $?
done
cat $O/rel.json $O/abl1.json $O/abl2.json
