#!/bin/bash
# bench lines under A/B knob settings (knobs build), any bench arguments:
#   CFGS="K=V K2=V;K=V" ARGS="--lstm --game SpaceInvaders-v0" TAG=... bash tools/r6/knob_ab_bench.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/${TAG:-r6kab}; mkdir -p $O
V=$ROOT/async-rl-tensorflow_amd/lib/var/knobs
make -C async-rl-tensorflow_amd/csrc -s -j16 OUT=$V/liba3c_hip.so OBJDIR=$V/obj EXTRA=-DA3C_KNOBS > $O/build.log 2>&1 || exit $?
IFS=';' read -ra LIST <<< "${CFGS:-A3C_CB_NWG=0}"
for rep in 1 2; do
for cfg in "${LIST[@]}"; do
  env A3C_LIB=$V/liba3c_hip.so $cfg timeout -k 10 300 python3 -u bench.py ${ARGS:-} --steps 20 --warmup 5 \
      --no-cpu-baseline --no-kernel-timing > $O/b.json 2>/dev/null || exit $?
  python3 -c "
import json
b=json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print('$cfg ${ARGS:-}', b['value'])" | tee -a $O/ab.txt
done
done
