set -o pipefail
V=async-rl-tensorflow_amd/lib/var
echo "### M1"
A3C_LIB=$V/wglog/liba3c_hip.so timeout -k 10 180 python3 tools/wglog.py 3 2>&1 | grep -v amdgpu.ids || exit 1
echo "### M2"
A3C_LIB=$V/wglog/liba3c_hip.so timeout -k 10 180 python3 tools/wglog.py 3 --frames84 2>&1 | grep -v amdgpu.ids || exit 1
