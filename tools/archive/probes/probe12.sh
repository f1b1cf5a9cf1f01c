# rollout sensitivity to co-resident work (hog build, measurement only)
export A3C_LIB=async-rl-tensorflow_amd/lib/var/hog/liba3c_hip.so
run() { echo "== type=$1 iters=$2"; A3C_HOG_TYPE=$1 A3C_HOG_ITERS=$2 timeout -k 10 120 python3 tools/span_timeline.py 300 2>&1 | grep -v amdgpu.ids || exit 1; }
run 5 1
run 0 600
run 1 600
run 2 600
run 3 1200
run 4 3000
run 5 500
run 6 2000
echo "== real backward"; timeout -k 10 120 python3 tools/span_timeline.py 300 2>&1 | grep -v amdgpu.ids
