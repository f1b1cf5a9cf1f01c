V=async-rl-tensorflow_amd/lib/var
AB_MODES=overlap AB_REPS=2 timeout -k 10 800 bash tools/ab.sh "A3C_LIB=$V/base/liba3c_hip.so" "A3C_LIB=$V/dly/liba3c_hip.so A3C_BWD_DELAY_US=0" "A3C_LIB=$V/dly/liba3c_hip.so A3C_BWD_DELAY_US=10" "A3C_LIB=$V/dly/liba3c_hip.so A3C_BWD_DELAY_US=20" "A3C_LIB=$V/dly/liba3c_hip.so A3C_BWD_DELAY_US=35" 2>&1 | grep -v amdgpu.ids
