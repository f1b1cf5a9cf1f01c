set -o pipefail
echo "### M1"
AB_MODES=overlap AB_REPS=2 timeout -k 10 900 bash tools/ab.sh "A3C_X=new" "A3C_GEMM_MULTI=1" "A3C_FOLD_LATE=1" "A3C_DWFC_LATE=1 A3C_FOLD_LATE=1" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### M2"
AB_MODES=overlap AB_REPS=2 AB_ARGS=--frames84 timeout -k 10 900 bash tools/ab.sh "A3C_X=new" "A3C_GEMM_MULTI=1" "A3C_FOLD_LATE=1" 2>&1 | grep -v amdgpu.ids || exit 1
