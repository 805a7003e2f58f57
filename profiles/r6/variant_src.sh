#!/bin/bash
# Build a variant libbre: the listed csrc/ sources recompiled with extra compile-time defines, the other
# objects from the default build, into csrc/build/variants/libbre_NAME.so.
# usage (repo root, CPU, after `make -C beam-radiance-estimate-pbrt_amd/csrc`):
#   profiles/r6/variant_src.sh NAME "-DDEF=1 ..." SRC.hip [SRC.hip ...]
set -o pipefail
HERE=$(cd "$(dirname "$0")/../.." && pwd)
CS=$HERE/beam-radiance-estimate-pbrt_amd/csrc
V=$CS/build/variants
NAME=$1
DEFS=$2
shift 2
mkdir -p "$V"
FLAGS="-std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math -fno-slp-vectorize -I$CS -I$HERE/include"
objs=$(ls "$CS"/build/*.o)
vobjs=""
for SRC in "$@"; do
  base=$(basename "$SRC" .hip)
  /opt/rocm/bin/hipcc $FLAGS $DEFS -c "$CS/$SRC" -o "$V/${base}_$NAME.o" || exit 1
  objs=$(echo "$objs" | grep -v "/$base.o$")
  vobjs="$vobjs $V/${base}_$NAME.o"
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$V/libbre_$NAME.so" $vobjs $objs || exit 1
echo "built $V/libbre_$NAME.so"
