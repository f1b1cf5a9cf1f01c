#!/bin/bash
# Quick GPU pass during development: selected GPU tests (PYTEST_K / PYTEST_FILES), then A/B bench configs ($@).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/quick; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit $rc; }
[ -n "$AB_KERS" ] && { AB_OVERLAP=1 timeout -k 10 100 python3 tools/fc_ab.py 2>&1 | grep -v amdgpu.ids || exit 1; }
[ $# -gt 0 ] && { AB_MODES=${AB_MODES:-overlap} AB_REPS=${AB_REPS:-2} bash tools/ab.sh "$@" || exit 1; }
exit 0
