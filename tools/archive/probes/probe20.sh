set -o pipefail
O=gpurun_out/probe20; mkdir -p $O
V=async-rl-tensorflow_amd/lib/var
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for L in "$V/base/liba3c_hip.so" ""; do
  A3C_LIB=$L timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --backend gloo --steps 100 --no-kernel-timing > $O/g2.json 2> $O/g2.err || { tail -5 $O/g2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/g2.json'));print('${L:-new}', d['value'])"
done
done
