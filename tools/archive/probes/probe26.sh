set -o pipefail
V=async-rl-tensorflow_amd/lib/var
A=$V/ablprep/liba3c_hip.so
echo "### M1 overlap: combinations of the backward-bound choices"
AB_MODES=overlap AB_REPS=3 timeout -k 10 900 bash tools/ab.sh "A3C_X=new" "A3C_GEMM_XCD=1" "A3C_GEMM_XCD=1 A3C_CB_LEAN=1" "A3C_LIB=$A A3C_GEMM_XCD=1" "A3C_LIB=$A A3C_GEMM_XCD=1 A3C_CB_LEAN=1" "A3C_LIB=$A A3C_GEMM_XCD=1 A3C_CB_LEAN=1 A3C_LATE_GO=0" 2>&1 | grep -v amdgpu.ids || exit 1
