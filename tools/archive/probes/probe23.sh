set -o pipefail
V=async-rl-tensorflow_amd/lib/var
O=gpurun_out/probe23; mkdir -p $O
bash tools/gpu_tests.sh > /dev/null 2>&1; rc=$?; tail -3 gpurun_out/tests/pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/tests/pytest.log | head -60; exit 1; }
for m in "overlap:" "overlap:--frames84" "sync:"; do
echo "### $m"
AB_MODES=${m%%:*} AB_REPS=3 AB_ARGS="${m#*:}" timeout -k 10 600 bash tools/ab.sh "A3C_LIB=$V/prev/liba3c_hip.so" "A3C_X=new" 2>&1 | grep -v amdgpu.ids || exit 1
done
echo "### 2 ranks (gloo, one GPU)"
for rep in 1 2; do
for L in "$V/prev/liba3c_hip.so" ""; do
  A3C_LIB=$L timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --backend gloo --steps 100 --no-kernel-timing > $O/g2.json 2> $O/g2.err || { tail -5 $O/g2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/g2.json'));print('${L:-new}', d['value'])"
done
done
