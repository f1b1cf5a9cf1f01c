set -o pipefail
V=async-rl-tensorflow_amd/lib/var
A3C_LIB=$V/cbp/liba3c_hip.so timeout -k 10 120 python3 tools/cb_phases.py 2>&1 | grep -v amdgpu.ids || exit 1
AB_MODES="overlap sync" AB_REPS=3 timeout -k 10 500 bash tools/ab.sh "A3C_LIB=$V/base/liba3c_hip.so" "A3C_X=new" 2>&1 | grep -v amdgpu.ids
