set -o pipefail
V=async-rl-tensorflow_amd/lib/var
bash tools/gpu_tests.sh > /dev/null 2>&1; rc=$?; tail -3 gpurun_out/tests/pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/tests/pytest.log | head -80; exit 1; }
A3C_CB_LEAN=1 A3C_LIB=$V/cbp/liba3c_hip.so timeout -k 10 200 python3 tools/cb_phases.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "### M2"
AB_MODES=overlap AB_REPS=3 AB_ARGS=--frames84 timeout -k 10 900 bash tools/ab.sh "A3C_LIB=$V/prev/liba3c_hip.so" "A3C_X=new" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### M1"
AB_MODES=overlap AB_REPS=2 timeout -k 10 900 bash tools/ab.sh "A3C_LIB=$V/prev/liba3c_hip.so" "A3C_X=new" 2>&1 | grep -v amdgpu.ids || exit 1
