cd ${GRAFT_REPO_ROOT:-.}
V=async-rl-tensorflow_amd/lib/var
timeout -k 10 120 python3 -u tools/fc_ab.py || exit 1
for n in s2 s8 s2w8 s4w8 s1w8; do A3C_LIB=$V/fc_$n/liba3c_hip.so timeout -k 10 120 python3 -u tools/fc_ab.py || exit 1; done
