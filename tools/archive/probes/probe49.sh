set -o pipefail
V=async-rl-tensorflow_amd/lib/var
echo "### M1: W prefetch depth of the 4-way K-split partial fc"
AB_MODES=overlap AB_REPS=3 AB_KT=k_fc_part timeout -k 10 900 bash tools/ab.sh "A3C_X=d4" "A3C_LIB=$V/d2/liba3c_hip.so" "A3C_LIB=$V/d8/liba3c_hip.so" 2>&1 | grep -v amdgpu.ids || exit 1
