V=async-rl-tensorflow_amd/lib/var
for r in 1 2; do
echo "== base"; A3C_LIB=$V/base/liba3c_hip.so timeout -k 10 120 python3 tools/span_timeline.py 300 2>&1 | grep -v amdgpu.ids | tail -1
echo "== new"; timeout -k 10 120 python3 tools/span_timeline.py 300 2>&1 | grep -v amdgpu.ids | tail -1
done
