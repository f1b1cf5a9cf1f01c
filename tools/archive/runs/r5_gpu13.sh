#!/bin/bash
# round 5: dl2 GEMM at its traffic floor (XCD-grouped order + ReLU-bit epilogue) vs the default, M1,
# 6 interleaved reps (knobs build); then the same pair under the PMC FETCH/WRITE passes
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
O=gpurun_out/r5g13; mkdir -p $O
K=async-rl-tensorflow_amd/lib/var/knobs/liba3c_hip.so
for rep in 1 2 3 4 5 6; do
  for cfg in "X=0" "A3C_GEMM_XCD=1 A3C_L2BITS=1"; do
    env A3C_LIB=$K $cfg timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-kernel-timing --steps 100 --min-seconds 1 > $O/b.json 2>$O/b.err || exit 1
    python3 -c "import json;d=json.load(open('$O/b.json'));print('$cfg', d['value'])"
  done
done
