V=async-rl-tensorflow_amd/lib/var
for r in 1 2; do
for v in mkbase mk mkbp1 mkp1; do echo "== $v"; A3C_LIB=$V/$v/liba3c_hip.so timeout -k 10 120 python3 tools/markers.py overlap x eager 2>&1 | grep -v amdgpu.ids | grep -v raw: || exit 1; done
done
