#!/bin/bash
# bench lines for compile-time variants of the library (knobs builds), any bench arguments:
#   VARS="name:-DX=1;base:" ARGS="--dqn-type nature" TAG=... bash tools/r6/var_bench.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/${TAG:-r6var}; mkdir -p $O
IFS=';' read -ra LIST <<< "${VARS:-base:}"
for v in "${LIST[@]}"; do
  name=${v%%:*}; defs=${v#*:}
  V=$ROOT/async-rl-tensorflow_amd/lib/var/$name
  make -C async-rl-tensorflow_amd/csrc -s -j16 OUT=$V/liba3c_hip.so OBJDIR=$V/obj EXTRA="-DA3C_KNOBS $defs" > $O/build_$name.log 2>&1 || exit $?
done
for rep in 1 2 3; do
for v in "${LIST[@]}"; do
  name=${v%%:*}
  A3C_LIB=$ROOT/async-rl-tensorflow_amd/lib/var/$name/liba3c_hip.so timeout -k 10 300 python3 -u bench.py ${ARGS:-} \
      --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing > $O/b.json 2>/dev/null || exit $?
  python3 -c "
import json
b=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$name ${ARGS:-}', b['value'])" | tee -a $O/ab.txt
done
done
