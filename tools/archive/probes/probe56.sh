set -o pipefail
PYTEST_ARGS=-k\ overlap A3C_GO_AT=2 bash tools/gpu_tests.sh > /dev/null 2>&1; rc=$?; tail -3 gpurun_out/tests/pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/tests/pytest.log | head -80; exit 1; }
echo "### M1: which rollout kernel carries the backward go"
AB_MODES=overlap AB_REPS=2 timeout -k 10 900 bash tools/ab.sh "A3C_GO_AT=0" "A3C_GO_AT=1" "A3C_GO_AT=2" 2>&1 | grep -v amdgpu.ids || exit 1
