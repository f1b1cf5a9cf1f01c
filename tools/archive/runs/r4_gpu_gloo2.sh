#!/bin/bash
# multi-rank GPU tests (two-phase exchange forced on gloo) + the 2- and 4-rank gloo bench rehearsal
set -o pipefail
mkdir -p gpurun_out/configs
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_multirank.py \
  > gpurun_out/mr_tests.log 2>&1 || { tail -40 gpurun_out/mr_tests.log; exit 1; }
tail -2 gpurun_out/mr_tests.log
for w in 2 4; do
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 --master-port 2953$w \
  bench.py --gpus $w --backend gloo --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing --min-seconds 0 > gpurun_out/configs/gloo$w.json 2> gpurun_out/configs/gloo$w.err || exit 2
python3 -c "import json;d=json.loads(open('gpurun_out/configs/gloo$w.json').read().strip().splitlines()[-1]);print('gloo$w', d['value'], d['ms_per_step'])"
done
