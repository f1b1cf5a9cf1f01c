set -o pipefail
echo "### M1: fc weight GEMM behind the conv backward (with the K-split fc)"
AB_MODES=overlap AB_REPS=3 timeout -k 10 900 bash tools/ab.sh "A3C_X=new" "A3C_DWFC_LATE=1" 2>&1 | grep -v amdgpu.ids || exit 1
