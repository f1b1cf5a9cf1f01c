set -o pipefail
bash tools/gpu_tests.sh > /dev/null 2>&1; rc=$?; tail -3 gpurun_out/tests/pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" gpurun_out/tests/pytest.log | head -80; exit 1; }
echo "### M1 overlap: bootstrap on the backward stream"
AB_MODES=overlap AB_REPS=3 timeout -k 10 900 bash tools/ab.sh "A3C_BOOT_BWD=0" "A3C_X=new" "A3C_CB_LEAN=1" 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 120 python3 tools/span_timeline.py 300 2>&1 | grep -v amdgpu.ids
