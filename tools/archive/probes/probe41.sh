set -o pipefail
echo "### M1"
AB_MODES=overlap AB_REPS=3 timeout -k 10 900 bash tools/ab.sh "A3C_CB_LEAN=0" "A3C_X=new" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### M2"
AB_MODES=overlap AB_REPS=3 AB_ARGS=--frames84 timeout -k 10 900 bash tools/ab.sh "A3C_LATE_GO=0" "A3C_X=new" 2>&1 | grep -v amdgpu.ids || exit 1
