V=async-rl-tensorflow_amd/lib/var
for r in 1 2; do
echo "== main"; timeout -k 10 120 python3 tools/span_timeline.py 300 2>&1 | grep -v amdgpu.ids || exit 1
echo "== newball"; A3C_LIB=$V/newball/liba3c_hip.so timeout -k 10 120 python3 tools/span_timeline.py 300 2>&1 | grep -v amdgpu.ids || exit 1
echo "== xcd"; A3C_GEMM_XCD=1 timeout -k 10 120 python3 tools/span_timeline.py 300 2>&1 | grep -v amdgpu.ids || exit 1
done
