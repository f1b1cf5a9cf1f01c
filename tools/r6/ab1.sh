#!/bin/bash
# Round 6 A/B (item 3 of VERDICT r5): what sits under rollout step 0 -- the fc weight GEMM in
# place (default), behind the conv backward (A3C_DWFC_LATE=1), or in its slab form (A3C_FC_WKS=0).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
O=gpurun_out/${TAG:-r6ab1}; mkdir -p $O
KB=$ROOT/async-rl-tensorflow_amd/lib/var/knobs
make -C async-rl-tensorflow_amd/csrc -s -j16 OUT=$KB/liba3c_hip.so OBJDIR=$KB/obj EXTRA=-DA3C_KNOBS > $O/build.log 2>&1 || exit $?
export A3C_LIB=$KB/liba3c_hip.so
AB_MODES=overlap AB_REPS=3 timeout -k 10 900 bash tools/ab.sh "A3C_X=0" "A3C_DWFC_LATE=1" "A3C_FC_WKS=0" > $O/ab.txt 2>&1
rc=$?; cat $O/ab.txt; exit $rc
