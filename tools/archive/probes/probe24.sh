set -o pipefail
V=async-rl-tensorflow_amd/lib/var
O=gpurun_out/probe24; mkdir -p $O
bash tools/gpu_tests.sh > /dev/null 2>&1; rc=$?; tail -3 gpurun_out/tests/pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/tests/pytest.log | head -60; exit 1; }
echo "### M1 overlap"
AB_MODES=overlap AB_REPS=3 timeout -k 10 600 bash tools/ab.sh "A3C_LIB=$V/prev/liba3c_hip.so" "A3C_X=new" "A3C_CB_LEAN=1" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### M2 overlap"
AB_MODES=overlap AB_REPS=2 AB_ARGS=--frames84 timeout -k 10 600 bash tools/ab.sh "A3C_LIB=$V/prev/liba3c_hip.so" "A3C_X=new" "A3C_LATE_GO=1" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### 2 ranks (gloo, one GPU)"
for rep in 1 2; do
for L in "$V/prev/liba3c_hip.so" ""; do
  A3C_LIB=$L timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --backend gloo --steps 100 --no-kernel-timing > $O/g2.json 2> $O/g2.err || { tail -5 $O/g2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/g2.json'));print('${L:-new}', d['value'])"
done
done
echo "### XCD GEMM order, backward-bound modes"
AB_MODES=sync AB_REPS=2 timeout -k 10 600 bash tools/ab.sh "A3C_X=new" "A3C_GEMM_XCD=1" 2>&1 | grep -v amdgpu.ids || exit 1
AB_MODES=overlap AB_REPS=2 AB_ARGS=--frames84 timeout -k 10 600 bash tools/ab.sh "A3C_X=new" "A3C_GEMM_XCD=1" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### no forward prep after warmup (ablation upper bound)"
AB_MODES=overlap AB_REPS=2 timeout -k 10 600 bash tools/ab.sh "A3C_X=new" "A3C_LIB=$V/ablprep/liba3c_hip.so" 2>&1 | grep -v amdgpu.ids || exit 1
AB_MODES=overlap AB_REPS=2 AB_ARGS=--frames84 timeout -k 10 600 bash tools/ab.sh "A3C_X=new" "A3C_LIB=$V/ablprep/liba3c_hip.so" 2>&1 | grep -v amdgpu.ids || exit 1
