#!/bin/bash
# round 4, first GPU call: the full GPU suite (race fix, multi-rank oracle checks), then the
# headline bench and the Hogwild shard-memory A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/r4_gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED rc=$?"; tail -40 gpurun_out/r4_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r4_gpu_tests.log
timeout -k 10 200 python bench.py --steps 20 > gpurun_out/r4_bench0.json 2> gpurun_out/r4_bench0.err || exit 2
for m in fine coarse; do
  timeout -k 10 120 python bench.py --steps 20 --envs 512 --update hogwild --hogwild-memory $m --no-cpu-baseline \
    > gpurun_out/r4_hog_$m.json 2> gpurun_out/r4_hog_$m.err || exit 3
done
python - <<'PY'
import json
for f in ('r4_bench0', 'r4_hog_fine', 'r4_hog_coarse'):
    d = json.load(open('gpurun_out/%s.json' % f))
    print(f, d['value'], (d.get('roofline') or {}).get('frac'))
PY
