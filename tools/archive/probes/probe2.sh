set -o pipefail
O=gpurun_out/probe2; mkdir -p $O
V=async-rl-tensorflow_amd/lib/var
AB_MODES=overlap AB_REPS=3 timeout -k 10 400 bash tools/ab.sh "A3C_X=0" "A3C_LIB=$V/nol1/liba3c_hip.so" > $O/ab.txt 2>&1 && \
A3C_ABL_BWD=1 A3C_LIB=$V/mk/liba3c_hip.so timeout -k 10 120 python3 tools/markers.py overlap x eager > $O/markers_rollout_alone.txt 2> $O/m.err
echo rc=$?
cat $O/ab.txt; head -8 $O/markers_rollout_alone.txt
