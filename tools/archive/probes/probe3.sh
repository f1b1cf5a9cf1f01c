# ablation timeline: what bounds the overlapped iteration (measurement only)
M=async-rl-tensorflow_amd/lib/var/mk/liba3c_hip.so
run() { echo "== $1"; shift; env "$@" timeout -k 10 120 python3 tools/markers.py overlap x eager 2>&1 | grep -v amdgpu.ids | grep -v raw: || exit 1; }
run base A3C_LIB=$M
run no_gemm A3C_LIB=$M A3C_ABL_GEMM=1
run no_cbwd A3C_LIB=$M A3C_ABL_CBWD=1
run no_gemm_cbwd A3C_LIB=$M A3C_ABL_GEMM=1 A3C_ABL_CBWD=1
run no_fc A3C_LIB=$M A3C_ABL_FC=1
