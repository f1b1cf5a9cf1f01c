#!/bin/bash
# a compile-time variant (knobs build with DEFS) through the nature parity tests, then
# whole-bench A/B against the plain knobs build: DEFS="-DX=1" KNOB="A3C_Y=1" TAG=... bash tools/r6/var_parity.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/${TAG:-r6vp}; mkdir -p $O
VB=$ROOT/async-rl-tensorflow_amd/lib/var/vbase; VV=$ROOT/async-rl-tensorflow_amd/lib/var/vvar
make -C async-rl-tensorflow_amd/csrc -s -j16 OUT=$VB/liba3c_hip.so OBJDIR=$VB/obj EXTRA="-DA3C_KNOBS" > $O/build_b.log 2>&1 || exit $?
make -C async-rl-tensorflow_amd/csrc -s -j16 OUT=$VV/liba3c_hip.so OBJDIR=$VV/obj EXTRA="-DA3C_KNOBS ${DEFS}" > $O/build_v.log 2>&1 || exit $?
A3C_LIB=$VV/liba3c_hip.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_nature.py -x -q --timeout 300 \
    --timeout-method thread -k "matches_oracle and not bench_shape" > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
for cfg in "b:A3C_X=0" "v:A3C_X=0" "v:${KNOB:-A3C_X=0}"; do
  lib=${cfg%%:*}; env_=${cfg#*:}; L=$VB; [ $lib = v ] && L=$VV
  env A3C_LIB=$L/liba3c_hip.so $env_ timeout -k 10 300 python3 -u bench.py --dqn-type nature --steps 20 --warmup 5 \
      --no-cpu-baseline > $O/b.json 2>/dev/null || exit $?
  python3 -c "
import json
b=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); k=b.get('kernels',{})
print('$lib $env_', b['value'], ' '.join('%s=%.1f'%(n[4:],v['avg_ms']*1e3) for n,v in k.items()))" | tee -a $O/ab.txt
done
done
