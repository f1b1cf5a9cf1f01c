#!/bin/bash
# Round 6: nature trunk parity on the GPU (small shapes first), then the NIPS engine tests.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/${TAG:-r6n1}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_nature.py -v -x --timeout 300 --timeout-method thread -k "not bench_shape" > $O/nat_small.log 2>&1
rc=$?; tail -30 $O/nat_small.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_headline_parity.py -v -x --timeout 300 --timeout-method thread -k "c2_headline_overlap_m1_matches or deterministic or fused" > $O/nips.log 2>&1
rc=$?; tail -8 $O/nips.log; exit $rc
