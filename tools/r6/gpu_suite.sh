#!/bin/bash
# Round 6: full GPU suite (no -x: every failure listed), then the default bench line and the
# spawned 2-rank gloo bench.  Test failures (rc 1) do not stop the chain; faults / timeouts do.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/${TAG:-r6a}; mkdir -p $O
(cat /proc/self/cgroup; echo; cat /sys/fs/cgroup/cpu.max; echo; nproc; python3 -c 'import os; print(len(os.sched_getaffinity(0)))'; env | grep -E 'OMP|MAX_JOBS') > $O/cgroup.txt 2>&1
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest.log 2>&1
rc=$?
tail -25 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
[ -n "$NO_BENCH" ] && exit $rc
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json | cut -c1-600
timeout -k 10 300 python3 -u bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --min-seconds 1 --no-kernel-timing > $O/bench_g2.json 2> $O/bench_g2.err || exit $?
cut -c1-300 $O/bench_g2.json
exit $rc
