set -o pipefail
O=gpurun_out/probe1; mkdir -p $O
timeout -k 10 120 python3 tools/host_ahead.py 400 > $O/host_ahead.json 2> $O/host_ahead.err && \
A3C_LIB=async-rl-tensorflow_amd/lib/var/mk/liba3c_hip.so timeout -k 10 120 python3 tools/markers.py overlap x eager > $O/markers.txt 2> $O/markers.err && \
A3C_LIB=async-rl-tensorflow_amd/lib/var/cbp/liba3c_hip.so timeout -k 10 120 python3 tools/cb_phases.py > $O/cbp.txt 2> $O/cbp.err
echo rc=$?
cat $O/host_ahead.json; tail -15 $O/markers.txt; cat $O/cbp.txt
