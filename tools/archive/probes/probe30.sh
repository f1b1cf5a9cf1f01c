set -o pipefail
V=async-rl-tensorflow_amd/lib/var
bash tools/gpu_tests.sh > /dev/null 2>&1; rc=$?; tail -3 gpurun_out/tests/pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/tests/pytest.log | head -80; exit 1; }
echo "### M1"
A3C_LIB=$V/wglog/liba3c_hip.so timeout -k 10 180 python3 tools/wglog.py 3 2>&1 | grep -v amdgpu.ids || exit 1
echo "### M2"
A3C_LIB=$V/wglog/liba3c_hip.so timeout -k 10 180 python3 tools/wglog.py 3 --frames84 2>&1 | grep -v amdgpu.ids || exit 1
