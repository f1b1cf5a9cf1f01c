V=async-rl-tensorflow_amd/lib/var
AB_MODES=overlap AB_REPS=2 timeout -k 10 800 bash tools/ab.sh "A3C_LIB=$V/base/liba3c_hip.so" "A3C_CB_NWG=192" "A3C_CB_NWG=160" "A3C_CB_NWG=128" "A3C_CB_NWG=224" "A3C_CB_NWG=256" 2>&1 | grep -v amdgpu.ids
