#!/bin/bash
# nature passes: fp32 vs bf16-term MFMA kernels, two / one LDS buffers (knobs build, per-pass us)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/${TAG:-r6bf}; mkdir -p $O
V=$ROOT/async-rl-tensorflow_amd/lib/var/knobs
make -C async-rl-tensorflow_amd/csrc -s -j16 OUT=$V/liba3c_hip.so OBJDIR=$V/obj EXTRA=-DA3C_KNOBS > $O/build.log 2>&1 || exit $?
K=$V/liba3c_hip.so
ALL=502   # bits NAT_C2F..NAT_C1W, the fp32-template passes
for cfg in "0 0" "$ALL 0" "$ALL $ALL"; do
  set -- $cfg
  echo "bf=$1 bf1=$2" >> $O/passes.txt
  A3C_LIB=$K A3C_NAT_BF=$1 A3C_NAT_BF1=$2 timeout -k 10 120 python3 -u tools/r6/nat_abl.py >> $O/passes.txt || exit $?
done
cat $O/passes.txt
