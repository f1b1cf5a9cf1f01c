set -o pipefail
echo "### M1 knobs in the 256-workgroup regime"
AB_MODES=overlap AB_REPS=2 timeout -k 10 1000 bash tools/ab.sh "A3C_X=new" "A3C_GEMM_MULTI=1" "A3C_GEMM_XCD=1" "A3C_DWFC_LATE=1" "A3C_FOLD_LATE=1" 2>&1 | grep -v amdgpu.ids || exit 1
echo "### M2 knobs"
AB_MODES=overlap AB_REPS=2 AB_ARGS=--frames84 timeout -k 10 900 bash tools/ab.sh "A3C_X=new" "A3C_FOLD_LATE=0 A3C_GEMM_MULTI=0 A3C_DWFC_LATE=1" "A3C_KERNEL_GO=0" 2>&1 | grep -v amdgpu.ids || exit 1
