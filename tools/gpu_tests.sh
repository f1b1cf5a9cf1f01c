#!/bin/bash
# GPU test pass on the box: pytest -m gpu (one process, per-test timeout), then a bench line.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/tests; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest.log 2>&1
rc=$?
tail -15 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err && cat $O/bench.json
