V=async-rl-tensorflow_amd/lib/var
AB_MODES=overlap AB_REPS=2 timeout -k 10 800 bash tools/ab.sh "A3C_X=main" "A3C_LIB=$V/pcb/liba3c_hip.so" "A3C_LIB=$V/phead/liba3c_hip.so" "A3C_LIB=$V/pscr/liba3c_hip.so" "A3C_LIB=$V/pfc/liba3c_hip.so" 2>&1 | grep -v amdgpu.ids || exit 1
for v in pcb phead pscr pfc; do echo "== $v"; A3C_LIB=$V/$v/liba3c_hip.so timeout -k 10 120 python3 tools/span_timeline.py 300 2>&1 | grep -v amdgpu.ids || exit 1; done
