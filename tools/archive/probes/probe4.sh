set -o pipefail
O=gpurun_out/probe4; mkdir -p $O
V=async-rl-tensorflow_amd/lib/var
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py tests/test_gpu_headline_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for v in cbpold cbp; do A3C_LIB=$V/$v/liba3c_hip.so timeout -k 10 120 python3 tools/cb_phases.py 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" || exit 1; done
AB_MODES=overlap AB_REPS=3 timeout -k 10 400 bash tools/ab.sh "A3C_LIB=$V/base/liba3c_hip.so" "A3C_X=new" 2>&1 | grep -v amdgpu.ids
