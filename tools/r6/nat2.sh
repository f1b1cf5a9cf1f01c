#!/bin/bash
# Round 6: nature trunk at the bench shape (parity), bench lines (overlap, sync), kernel trace.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/${TAG:-r6n2}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_nature.py -v -x --timeout 600 --timeout-method thread -k "bench_shape" > $O/nat_bench_shape.log 2>&1
rc=$?; tail -6 $O/nat_bench_shape.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -u bench.py --dqn-type nature --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_nat.json 2> $O/bench_nat.err || exit $?
cut -c1-400 $O/bench_nat.json
timeout -k 10 300 python3 -u bench.py --dqn-type nature --update sync --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing > $O/bench_nat_sync.json 2> $O/bench_nat_sync.err || exit $?
cut -c1-200 $O/bench_nat_sync.json
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --dqn-type nature --steps 50 --no-cpu-baseline --no-kernel-timing --min-seconds 1 > $O/trace.log 2>&1 || exit $?
find $O/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
head -20 $O/kernel_stats.csv | cut -c1-200
exit $rc
