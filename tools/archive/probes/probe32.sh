set -o pipefail
A3C_GEMM_WGS=256 bash tools/gpu_tests.sh > /dev/null 2>&1; rc=$?; tail -3 gpurun_out/tests/pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/tests/pytest.log | head -80; exit 1; }
echo "### M1"
AB_MODES=overlap AB_REPS=2 timeout -k 10 900 bash tools/ab.sh "A3C_GEMM_WGS=0" "A3C_GEMM_WGS=256" "A3C_GEMM_WGS=512" "A3C_GEMM_WGS=128" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### M2"
AB_MODES=overlap AB_REPS=2 AB_ARGS=--frames84 timeout -k 10 900 bash tools/ab.sh "A3C_GEMM_WGS=0" "A3C_GEMM_WGS=256" "A3C_GEMM_WGS=512" "A3C_GEMM_WGS=128" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### dW_fc GEMM behind the conv backward"
AB_MODES=overlap AB_REPS=2 timeout -k 10 900 bash tools/ab.sh "A3C_DWFC_LATE=0" "A3C_DWFC_LATE=1" "A3C_DWFC_LATE=1 A3C_GEMM_WGS=256" 2>&1 | grep -v amdgpu.ids || exit 1
AB_MODES=overlap AB_REPS=2 AB_ARGS=--frames84 timeout -k 10 900 bash tools/ab.sh "A3C_DWFC_LATE=0" "A3C_DWFC_LATE=1" 2>&1 | grep -v amdgpu.ids || exit 1
