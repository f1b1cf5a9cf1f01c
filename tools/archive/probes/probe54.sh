set -o pipefail
echo "### M1: cross-stream ordering by events vs wait-value"
AB_MODES=overlap AB_REPS=2 timeout -k 10 900 bash tools/ab.sh "A3C_X=new" "A3C_WAIT_VALUE=0" 2>&1 | grep -v amdgpu.ids || exit 1
