set -o pipefail
O=gpurun_out/probe18; mkdir -p $O
V=async-rl-tensorflow_amd/lib/var
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_headline_parity.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for args in "--frames84" ""; do
echo "### $args"
AB_MODES=overlap AB_REPS=3 AB_ARGS="$args" timeout -k 10 600 bash tools/ab.sh "A3C_LIB=$V/base/liba3c_hip.so" "A3C_X=new" 2>&1 | grep -v amdgpu.ids || exit 1
done
