#!/bin/bash
# Other BASELINE configs on one GPU + a 2-rank gloo rehearsal of the multi-GPU bench path.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/configs; mkdir -p $O
run() { name=$1; shift; timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-kernel-timing "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('%-12s %12.1f' % ('$name', d['value']))"; }
run default && run m2_frames84 --frames84 && run sync --update sync && run c3_breakout --game Breakout-v0 && run c4_512 --envs 512 && \
run c4_hogwild --envs 512 --update hogwild && run c5_lstm --lstm --game SpaceInvaders-v0 && run e1024 --envs 1024 && \
run q_sync --algo q --n-step 32 --update sync && run q_overlap --algo q --n-step 32 && \
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing --min-seconds 0 > $O/gloo2.json 2> $O/gloo2.err && \
python3 -c "import json;d=json.loads(open('$O/gloo2.json').read().strip().splitlines()[-1]);print('gloo2 (2 ranks, 1 GPU) %.1f' % d['value'], d['config']['parallelism'])"
