set -o pipefail
A3C_GEMM_BIG_MULTI=1 bash tools/gpu_tests.sh > /dev/null 2>&1; rc=$?; tail -3 gpurun_out/tests/pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/tests/pytest.log | head -80; exit 1; }
echo "### M2: single-launch GEMMs with 128x128 dl2 tiles"
AB_MODES=overlap AB_REPS=3 AB_ARGS=--frames84 timeout -k 10 900 bash tools/ab.sh "A3C_X=new" "A3C_GEMM_BIG_MULTI=1" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### sync"
AB_MODES=sync AB_REPS=2 timeout -k 10 900 bash tools/ab.sh "A3C_X=new" 2>&1 | grep -v amdgpu.ids || exit 1
