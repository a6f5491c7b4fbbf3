#!/bin/bash
# A/B build: libgtr_hip.so with ONE source file recompiled under extra defines, linked with
# the default build's other objects -> gat-recommendation_amd/build/var_NAME/libgtr_hip.so
# (select at run time with GTR_LIB=...).  usage: build_variant.sh NAME SRC "-DFOO=1 ..."
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; SRC=$2; DEFS=$3
B=$ROOT/gat-recommendation_amd/build
OUT=$B/var_$NAME
mkdir -p "$OUT"
cd "$ROOT/gat-recommendation_amd/csrc"
make -s -j8 >/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -I../../include $DEFS \
  -c $SRC.hip -o "$OUT/$SRC.o"
objs=""
for o in "$B"/*.o; do
  n=$(basename "$o")
  if [ "$n" = "$SRC.o" ]; then objs="$objs $OUT/$SRC.o"; else objs="$objs $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libgtr_hip.so" $objs
echo "$OUT/libgtr_hip.so ($SRC.hip $DEFS)"
