set -o pipefail
O=gpurun_out/probe9; mkdir -p $O
V=async-rl-tensorflow_amd/lib/var
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py tests/test_gpu_headline_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
AB_MODES="overlap sync" AB_REPS=3 timeout -k 10 800 bash tools/ab.sh "A3C_LIB=$V/base/liba3c_hip.so" "A3C_X=new" "A3C_GEMM_XCD=0" 2>&1 | grep -v amdgpu.ids || exit 1
bash tools/profile_round.sh r3v1 > $O/prof.log 2>&1; tail -3 $O/prof.log
