#!/bin/bash
# Ablation timeline (marker build, measurement only -- results are not valid training):
# baseline, no fc, no conv backward, no backward at all, L2-resident frames.
M=async-rl-tensorflow_amd/lib/var/mk/liba3c_hip.so
F=async-rl-tensorflow_amd/lib/var/mkf/liba3c_hip.so
run() { echo "== $1"; shift; env "$@" timeout -k 10 120 python3 tools/markers.py ${MODE:-overlap} 2>&1 | grep -v amdgpu.ids || exit 1; }
run base A3C_LIB=$M
run no_fc A3C_LIB=$M A3C_ABL_FC=1
run no_cbwd A3C_LIB=$M A3C_ABL_CBWD=1
run no_bwd A3C_LIB=$M A3C_ABL_BWD=1
run l2_frames A3C_LIB=$F
run no_bwd_l2_frames A3C_LIB=$F A3C_ABL_BWD=1
MODE=sync run sync_base A3C_LIB=$M
MODE=sync run sync_no_fc A3C_LIB=$M A3C_ABL_FC=1
MODE=sync run sync_l2_frames A3C_LIB=$F
