#!/bin/bash
# round-4 close: the full GPU suite, smoke(), the headline bench (with the CPU baseline) and the
# other BASELINE configs (tools/configs_bench.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  > gpurun_out/r4_final_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 gpurun_out/r4_final_tests.log; exit 1; }
tail -3 gpurun_out/r4_final_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_final_smoke.log 2>&1 || { tail -20 gpurun_out/r4_final_smoke.log; exit 2; }
tail -1 gpurun_out/r4_final_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r4_final_bench.json 2> gpurun_out/r4_final_bench.err || { tail -20 gpurun_out/r4_final_bench.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/r4_final_bench.json'));print('bench', d['value'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 1500 bash tools/configs_bench.sh
