set -o pipefail
V=async-rl-tensorflow_amd/lib/var
O=gpurun_out/probe25; mkdir -p $O
bash tools/gpu_tests.sh > /dev/null 2>&1; rc=$?; tail -3 gpurun_out/tests/pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/tests/pytest.log | head -60; exit 1; }
for m in "overlap:" "overlap:--frames84"; do
echo "### $m"
AB_MODES=${m%%:*} AB_REPS=3 AB_ARGS="${m#*:}" timeout -k 10 600 bash tools/ab.sh "A3C_LIB=$V/head/liba3c_hip.so" "A3C_X=new" 2>&1 | grep -v amdgpu.ids || exit 1
done
