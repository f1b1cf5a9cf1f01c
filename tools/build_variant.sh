#!/bin/bash
# Kernel A/B builds: tools/build_variant.sh NAME "-DMACRO=V ..." [source.hip]
# -> async-rl-tensorflow_amd/lib/var/NAME/liba3c_hip.so (select with A3C_LIB=... in tools/ab.sh)
# source: a csrc file name, or a path to another version of it (e.g. from git show)
set -e
NAME=$1; DEFS=$2; SRC=${3:-net_bwd.hip}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/async-rl-tensorflow_amd/csrc
make -C "$C" -s
OUT=$ROOT/async-rl-tensorflow_amd/lib/var/$NAME
mkdir -p "$OUT"
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5"
case "$SRC" in */*) SP=$SRC; SRC=$(basename "$SRC");; *) SP=$C/$SRC;; esac
/opt/rocm/bin/hipcc $FL -I"$C" $DEFS -c "$SP" -o "$OUT/${SRC%.hip}.o"
OBJS=""
for o in "$ROOT"/async-rl-tensorflow_amd/lib/obj/*.o; do
  b=$(basename "$o")
  if [ "$b" = "${SRC%.hip}.o" ]; then OBJS="$OBJS $OUT/$b"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -mcode-object-version=5 $OBJS -o "$OUT/liba3c_hip.so"
echo "$OUT/liba3c_hip.so"
