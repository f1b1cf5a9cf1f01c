V=async-rl-tensorflow_amd/lib/var
AB_MODES=overlap AB_REPS=3 timeout -k 10 800 bash tools/ab.sh "A3C_LIB=$V/base/liba3c_hip.so" "A3C_X=new" "A3C_LIB=$V/noprep/liba3c_hip.so" "A3C_LIB=$V/bnoprep/liba3c_hip.so" 2>&1 | grep -v amdgpu.ids
