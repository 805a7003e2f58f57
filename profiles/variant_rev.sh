#!/bin/bash
# Build libbre_NAME.so with bre_gather.hip taken from git revision REV (the other objects from the
# current build): a same-box A/B baseline for a kernel change.
# usage (repo root, CPU): profiles/variant_rev.sh NAME REV   (needs `make -C .../csrc` first)
set -o pipefail
HERE=$(cd "$(dirname "$0")/.." && pwd)
CS=$HERE/beam-radiance-estimate-pbrt_amd/csrc
V=$CS/build/variants
NAME=$1
REV=$2
mkdir -p "$V/src_$NAME"
git -C "$HERE" show "$REV:beam-radiance-estimate-pbrt_amd/csrc/bre_gather.hip" > "$V/src_$NAME/bre_gather.hip" || exit 1
FLAGS="-std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math -fno-slp-vectorize -I$CS -I$HERE/include"
/opt/rocm/bin/hipcc $FLAGS -c "$V/src_$NAME/bre_gather.hip" -o "$V/bre_gather_$NAME.o" || exit 1
objs=$(ls "$CS"/build/*.o | grep -v bre_gather.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$V/libbre_$NAME.so" "$V/bre_gather_$NAME.o" $objs || exit 1
echo "built $V/libbre_$NAME.so"
