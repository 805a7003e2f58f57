#!/bin/bash
# Profiles a bench workload on one MI355X (run via gpurun from the repo root).
# Pass 1: kernel trace + stats.  Passes 2/3: HBM traffic counters, one TCC counter per pass
# (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950; MI355X_MICROARCH.md §rocprofv3).
# usage: profiles/run_profiles.sh OUTDIR [bench args...]   (default bench args: --steps 5 --warmup 1)
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
shift || true
ARGS=("$@")
if [ ${#ARGS[@]} -eq 0 ]; then ARGS=(--steps 5 --warmup 1); fi
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py "${ARGS[@]}" --no-cpu --no-diag > "$OUT/bench_trace.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- \
    python3 bench.py "${ARGS[@]}" --no-cpu --no-diag > "$OUT/bench_fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- \
    python3 bench.py "${ARGS[@]}" --no-cpu --no-diag > "$OUT/bench_write.log" 2>&1
python3 profiles/summarize.py "$OUT" "$OUT/profile_summary.json" > "$OUT/summary.log"
cp "$OUT/trace/run_kernel_stats.csv" "$OUT/kernel_stats.csv"
echo "profiles done"
