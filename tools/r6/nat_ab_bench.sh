#!/bin/bash
# nature bench lines under A/B knob settings (knobs build): CFGS="K=V K2=V;K=V" TAG=... bash tools/r6/nat_ab_bench.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/${TAG:-r6ab}; mkdir -p $O
V=$ROOT/async-rl-tensorflow_amd/lib/var/knobs
make -C async-rl-tensorflow_amd/csrc -s -j16 OUT=$V/liba3c_hip.so OBJDIR=$V/obj EXTRA=-DA3C_KNOBS > $O/build.log 2>&1 || exit $?
IFS=';' read -ra LIST <<< "${CFGS:-A3C_NAT_BF=0}"
for rep in 1 2; do
for cfg in "${LIST[@]}"; do
  env A3C_LIB=$V/liba3c_hip.so $cfg timeout -k 10 300 python3 -u bench.py --dqn-type nature --steps 20 --warmup 5 \
      --no-cpu-baseline ${BENCH_ARGS:-} > $O/b.json 2>/dev/null || exit $?
  python3 -c "
import json,sys
b=json.loads(open('$O/b.json').read().strip().splitlines()[-1])
k=b.get('kernels',{})
print('$cfg', b['value'], ' '.join('%s=%.1f'%(n[4:],v['avg_ms']*1e3) for n,v in k.items()))" | tee -a $O/ab.txt
done
done
