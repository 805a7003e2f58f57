#!/bin/bash
# One SQ-counter pass (8 SQ counters max per pass on gfx950) over one C2 iteration of the bench.
# usage: profiles/pmc_sq.sh OUTDIR [bench args...]
set -e
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p "$OUT"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU \
    --kernel-trace --output-format csv -d "$OUT/sq" -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-diag "$@" > "$OUT/sq.log" 2>&1
echo "pmc done"
