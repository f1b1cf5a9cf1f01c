#!/bin/bash
# (1) M1 A/B of the fc weight GEMM's XCD-grouped order (the knob now reaches the launch);
# (2) per-kernel stats of C5 (LSTM) with the round-3 and round-4 builds, to find its regression.
set -o pipefail
mkdir -p gpurun_out
AB_MODES=overlap AB_REPS=3 timeout -k 10 600 bash tools/ab.sh "A3C_WKS_XCD=1" "A3C_WKS_XCD=0" 2>&1 | grep -v amdgpu.ids || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R3=$PWD/async-rl-tensorflow_amd/lib/var/r3/liba3c_hip.so
for v in r4 r3; do
  if [ $v = r3 ]; then export A3C_LIB=$R3; else unset A3C_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lstm_$v -o lp -- \
    python3 bench.py --lstm --game SpaceInvaders-v0 --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/lstm_$v.log 2>&1 || { tail -20 gpurun_out/lstm_$v.log; exit 2; }
  grep '"metric"' gpurun_out/lstm_$v.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v', d['value'])"
done
