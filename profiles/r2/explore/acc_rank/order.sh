#!/bin/bash
# r2: summation order of the rank accumulation on fixed beams/segments (seg_rgb hashes): production,
# pure per-run RMW (rmw64), pure rank RMW (rk64), rank + atomics (rk8, twice)
set -o pipefail
V=beam-radiance-estimate-pbrt_amd/csrc/build/variants
H=profiles/r2/explore/acc_rank/seghash.py
for l in beam-radiance-estimate-pbrt_amd/libbre.so beam-radiance-estimate-pbrt_amd/libbre.so $V/libbre_rmw64.so $V/libbre_rk64.so $V/libbre_rk8.so $V/libbre_rk8.so; do
  echo -n "$(basename $l) "; BRE_LIBRARY=$l timeout -k 10 120 python -u $H || exit 1
done
