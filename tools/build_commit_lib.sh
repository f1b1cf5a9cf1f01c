#!/bin/bash
# Build liba3c_hip.so of an earlier commit for same-box A/B runs (A3C_LIB=...):
#   tools/build_commit_lib.sh COMMIT NAME  ->  async-rl-tensorflow_amd/lib/var/NAME/liba3c_hip.so
set -e
C=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=/tmp/a3c_commit_$NAME
rm -rf "$T"; mkdir -p "$T"
git -C "$ROOT" archive "$C" async-rl-tensorflow_amd/csrc include | tar -x -C "$T"
OUT=$ROOT/async-rl-tensorflow_amd/lib/var/$NAME
mkdir -p "$OUT"
make -C "$T/async-rl-tensorflow_amd/csrc" -s -j8 OUT="$OUT/liba3c_hip.so" OBJDIR="$T/obj"
echo "$OUT/liba3c_hip.so"
