#!/bin/bash
# M1 upper bounds (measurement only): a markers build with and without the fc / head weight and
# dl2 GEMMs (A3C_ABL_GEMM: results wrong, time only), two interleaved reps
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/${TAG:-r6m1abl}; mkdir -p $O
V=$ROOT/async-rl-tensorflow_amd/lib/var/markers
make -C async-rl-tensorflow_amd/csrc -s -j16 OUT=$V/liba3c_hip.so OBJDIR=$V/obj EXTRA="-DA3C_KNOBS -DA3C_MARKERS" > $O/build.log 2>&1 || exit $?
for rep in 1 2; do
for cfg in "A3C_X=0" "A3C_ABL_GEMM=1"; do
  env A3C_LIB=$V/liba3c_hip.so $cfg timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      --no-kernel-timing > $O/b.json 2>/dev/null || exit $?
  python3 -c "
import json
b=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$cfg', b['value'])" | tee -a $O/ab.txt
done
done
