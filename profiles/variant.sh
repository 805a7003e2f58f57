#!/bin/bash
# Build a profiling variant of libbre with extra compile-time defines for bre_gather.hip
# (e.g. -DBRE_ABLATE=2, -DBRE_PHASE_TIMING=1) into csrc/build/variants/libbre_NAME.so.
# usage (repo root, CPU): profiles/variant.sh NAME "-DDEF=1 ..."   (needs `make -C .../csrc` first)
set -o pipefail
HERE=$(cd "$(dirname "$0")/.." && pwd)
CS=$HERE/beam-radiance-estimate-pbrt_amd/csrc
V=$CS/build/variants
NAME=$1
DEFS=$2
mkdir -p "$V"
FLAGS="-std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math ${VARIANT_FLAGS:--fno-slp-vectorize} -I$CS -I$HERE/include"
/opt/rocm/bin/hipcc $FLAGS $DEFS -c "$CS/bre_gather.hip" -o "$V/bre_gather_$NAME.o" || exit 1
objs=$(ls "$CS"/build/*.o | grep -v bre_gather.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$V/libbre_$NAME.so" "$V/bre_gather_$NAME.o" $objs || exit 1
echo "built $V/libbre_$NAME.so"
