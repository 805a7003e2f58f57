#!/bin/bash
# Phase timing (profiles/phase_timing.py) of every variant library given (via gpurun).
# usage: profiles/phase_variants.sh OUTDIR NAME...   (csrc/build/variants/libbre_NAME.so)
set -o pipefail
OUT=$1
shift
mkdir -p "$OUT"
for n in "$@"; do
  BRE_LIBRARY=beam-radiance-estimate-pbrt_amd/csrc/build/variants/libbre_$n.so timeout -k 10 200 \
      python -u profiles/phase_timing.py ${PHASE_ARGS:-0 8} > "$OUT/$n.log" 2>&1 || { echo "$n failed"; tail -n 20 "$OUT/$n.log"; exit 1; }
  echo "== $n"; grep iteration "$OUT/$n.log"
done
