#!/bin/bash
# Build libbre_NAME.so from the whole native tree (csrc + include) at git revision REV: a same-box A/B
# baseline for a change outside bre_gather.hip.
# usage (repo root, CPU): profiles/variant_tree.sh NAME REV
set -o pipefail
HERE=$(cd "$(dirname "$0")/.." && pwd)
V=$HERE/beam-radiance-estimate-pbrt_amd/csrc/build/variants
NAME=$1
REV=$2
T=$V/tree_$NAME
rm -rf "$T" && mkdir -p "$T"
git -C "$HERE" archive "$REV" beam-radiance-estimate-pbrt_amd/csrc include | tar -x -C "$T" || exit 1
make -C "$T/beam-radiance-estimate-pbrt_amd/csrc" -j8 OUT="$V/libbre_$NAME.so" OBJDIR="$T/obj" > "$T/build.log" 2>&1 \
    || { tail -n 20 "$T/build.log"; exit 1; }
rm -rf "$T/obj"
echo "built $V/libbre_$NAME.so"
