#!/bin/bash
# per-kernel stats of 1024 envs with the round-3 and the final round-4 build
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R3=$PWD/async-rl-tensorflow_amd/lib/var/r3/liba3c_hip.so
for v in r4 r3; do
  if [ $v = r3 ]; then export A3C_LIB=$R3; else unset A3C_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/e1024_$v -o lp -- \
    python3 bench.py --envs 1024 --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/e1024_$v.log 2>&1 || { tail -20 gpurun_out/e1024_$v.log; exit 2; }
  grep '"metric"' gpurun_out/e1024_$v.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v', d['value'])"
done
