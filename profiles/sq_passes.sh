#!/bin/bash
# SQ (issue / wait) counter passes over a short bench run, one rocprofv3 pass per counter group
# (8 SQ + 2 GRBM counters at most per pass on gfx950, MI355X_MICROARCH.md §rocprofv3 PMC slots).
# usage (repo root, via gpurun): profiles/sq_passes.sh OUTDIR [bench args...]
#   default bench args: --steps 2 --warmup 0 (C2 iterations 0 and 1)
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/sq}
shift || true
ARGS=("$@")
if [ ${#ARGS[@]} -eq 0 ]; then ARGS=(--steps 2 --warmup 0); fi
mkdir -p "$OUT"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
    SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
    -d "$OUT/sqa" -o run -- python3 bench.py "${ARGS[@]}" --no-cpu --no-diag > "$OUT/sqa.log" 2>&1 || { echo "pass A failed"; tail -n 20 "$OUT/sqa.log"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
    SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
    -d "$OUT/sqb" -o run -- python3 bench.py "${ARGS[@]}" --no-cpu --no-diag > "$OUT/sqb.log" 2>&1 || { echo "pass B failed"; tail -n 20 "$OUT/sqb.log"; exit 1; }
python3 profiles/summarize_sq.py "$OUT" "$OUT/sq_summary.json"
echo "sq passes done"
