#!/bin/bash
# Round 6 perf call 1: per-workgroup timeline of the final-r5 build (which backward kernel runs
# beside each rollout step) and the two-group throughput probe.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/${TAG:-r6p1}; mkdir -p $O
V=$ROOT/async-rl-tensorflow_amd/lib/var/wglog
timeout -k 10 120 python3 -u tools/r6/two_groups_probe.py 2 > $O/two_groups.json 2> $O/two_groups.err || exit $?
cat $O/two_groups.json
make -C async-rl-tensorflow_amd/csrc -s -j16 OUT=$V/liba3c_hip.so OBJDIR=$V/obj EXTRA=-DA3C_WGLOG > $O/build.log 2>&1 || exit $?
for i in 1 2; do
  A3C_LIB=$V/liba3c_hip.so timeout -k 10 120 python3 -u tools/wglog.py 3 > $O/wglog_$i.txt 2> $O/wglog_$i.err || exit $?
done
cat $O/wglog_1.txt
