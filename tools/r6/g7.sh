#!/bin/bash
# Round 6: drop-in Network tests (nature per-op kernels, same-activation gradient bar), then the
# two-group throughput probe with enough hardware queues for its streams.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/${TAG:-r6g7}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dropin.py -v --timeout 300 --timeout-method thread > $O/dropin.log 2>&1
rc=$?; tail -8 $O/dropin.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python3 -u tools/r6/two_groups_probe.py 2 > $O/two_groups_q8.json 2> $O/two_groups_q8.err || exit $?
cat $O/two_groups_q8.json
exit $rc
