#!/bin/bash
# Kernel A/B builds: tools/build_variant.sh NAME "-DMACRO=V ..." [source.hip]
# -> async-rl-tensorflow_amd/lib/var/NAME/liba3c_hip.so (select with A3C_LIB=... in tools/ab.sh)
# source: a csrc file name, or a path to another version of it (e.g. from git show)
# Variants are built with -DA3C_KNOBS over a knobs build of the other sources (lib/var/knobs), so
# the A/B environment knobs (A3C_AB_KNOB, a3c_common.h) are live in them; a release build ignores them.
# NAME=knobs alone builds that library: tools/build_variant.sh knobs ""
set -e
NAME=$1; DEFS=$2; SRC=${3:-net_bwd.hip}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/async-rl-tensorflow_amd/csrc
KB=$ROOT/async-rl-tensorflow_amd/lib/var/knobs
make -C "$C" -s OUT="$KB/liba3c_hip.so" OBJDIR="$KB/obj" EXTRA=-DA3C_KNOBS
[ "$NAME" = knobs ] && { echo "$KB/liba3c_hip.so"; exit 0; }
OUT=$ROOT/async-rl-tensorflow_amd/lib/var/$NAME
mkdir -p "$OUT"
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -DA3C_KNOBS"
case "$SRC" in */*) SP=$SRC; SRC=$(basename "$SRC");; *) SP=$C/$SRC;; esac
/opt/rocm/bin/hipcc $FL -I"$C" $DEFS -c "$SP" -o "$OUT/${SRC%.hip}.o"
OBJS=""
for o in "$KB"/obj/*.o; do
  b=$(basename "$o")
  if [ "$b" = "${SRC%.hip}.o" ]; then OBJS="$OBJS $OUT/$b"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -mcode-object-version=5 $OBJS -o "$OUT/liba3c_hip.so"
echo "$OUT/liba3c_hip.so"
