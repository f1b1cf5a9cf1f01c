#!/bin/bash
# Round 6: nature trunk parity (all) + bench line with per-pass timings.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/${TAG:-r6n3}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_nature.py -v -x --timeout 600 --timeout-method thread > $O/nat.log 2>&1
rc=$?; tail -12 $O/nat.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 -u bench.py --dqn-type nature --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_nat.json 2> $O/bench_nat.err || exit $?
python3 -c "
import json
b=json.loads([l for l in open('$O/bench_nat.json') if l.startswith('{')][0])
print(b['value'], b['ms_per_step'], b['roofline']['kernel'], b['roofline']['frac'])
for k,v in b['kernels'].items(): print(k, v['avg_ms'], v['achieved'], v['share'])
"
