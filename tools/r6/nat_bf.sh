#!/bin/bash
# nature passes per-pass us (a3c_engine_time_kernel) under A/B knob settings (knobs build):
#   CFGS="A3C_NAT_BF=0;A3C_NAT_BF=502 A3C_NAT_BF1=502" TAG=... bash tools/r6/nat_bf.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/${TAG:-r6bf}; mkdir -p $O
V=$ROOT/async-rl-tensorflow_amd/lib/var/knobs
make -C async-rl-tensorflow_amd/csrc -s -j16 OUT=$V/liba3c_hip.so OBJDIR=$V/obj EXTRA=-DA3C_KNOBS > $O/build.log 2>&1 || exit $?
IFS=';' read -ra LIST <<< "${CFGS:-A3C_NAT_BF=0}"
for cfg in "${LIST[@]}"; do
  echo "$cfg" >> $O/passes.txt
  env A3C_LIB=$V/liba3c_hip.so $cfg timeout -k 10 120 python3 -u tools/r6/nat_abl.py >> $O/passes.txt || exit $?
done
cat $O/passes.txt
