#!/bin/bash
# same-box A/B of the round-3 and round-4 builds on the configs whose round-4 column read lower
# (C5 LSTM, 1024 envs) plus C4 512 envs, interleaved.
set -o pipefail
mkdir -p gpurun_out
R3=A3C_LIB=$PWD/async-rl-tensorflow_amd/lib/var/r3/liba3c_hip.so
for args in "--lstm --game SpaceInvaders-v0" "--envs 1024" "--envs 512"; do
  AB_MODES=overlap AB_REPS=2 AB_ARGS="$args" timeout -k 10 600 bash tools/ab.sh "A3C_X=r4" "$R3" 2>&1 | sed "s|^|[$args] |" || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lstmprof -o lp -- \
  python3 bench.py --lstm --game SpaceInvaders-v0 --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/lstmprof.log 2>&1 || { tail -20 gpurun_out/lstmprof.log; exit 2; }
find gpurun_out/lstmprof -name '*stats*'
