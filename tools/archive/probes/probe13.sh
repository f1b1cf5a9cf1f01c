set -o pipefail
O=gpurun_out/probe13; mkdir -p $O
V=async-rl-tensorflow_amd/lib/var
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py tests/test_gpu_headline_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
A3C_LIB=$V/cbp/liba3c_hip.so timeout -k 10 120 python3 tools/cb_phases.py 2>&1 | grep -v amdgpu.ids || exit 1
AB_MODES="overlap sync" AB_REPS=3 timeout -k 10 800 bash tools/ab.sh "A3C_LIB=$V/base/liba3c_hip.so" "A3C_X=new" 2>&1 | grep -v amdgpu.ids || exit 1
bash tools/pmc_lds.sh split > /dev/null 2>&1; grep conv_bwd gpurun_out/lds_split/summary.txt
