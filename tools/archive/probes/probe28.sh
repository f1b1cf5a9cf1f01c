set -o pipefail
echo "### M1 overlap: bootstrap on the backward stream, early go"
AB_MODES=overlap AB_REPS=2 timeout -k 10 900 bash tools/ab.sh "A3C_BOOT_BWD=0" "A3C_LATE_GO=0" "A3C_LATE_GO=0 A3C_CB_LEAN=1" "A3C_BOOT_BWD=0 A3C_LATE_GO=0" 2>&1 | grep -v amdgpu.ids || exit 1
A3C_LATE_GO=0 timeout -k 10 120 python3 tools/span_timeline.py 300 2>&1 | grep -v amdgpu.ids
A3C_BOOT_BWD=0 timeout -k 10 120 python3 tools/span_timeline.py 300 2>&1 | grep -v amdgpu.ids
