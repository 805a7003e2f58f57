#!/bin/bash
# Round 6 study 7 (via gpurun): the tile kernel's tail (profiles/r6/wave_times.py on a BRE_WAVE_TIMES build).
set -o pipefail
OUT=$1; mkdir -p "$OUT"
export TMPDIR=/tmp
L=beam-radiance-estimate-pbrt_amd/csrc/build/variants/libbre_wt.so
for cfg in "0 0 1" "8 0 1" "15 0 1" "0 0 8" "8 0 8" "15 0 8" "8 5 8"; do
  BRE_LIBRARY=$L timeout -k 10 200 python3 -u profiles/r6/wave_times.py $cfg >> "$OUT/wave_times.txt" 2>&1 \
      || { tail -n 20 "$OUT/wave_times.txt"; exit 1; }
done
cat "$OUT/wave_times.txt"
