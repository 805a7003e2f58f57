#!/bin/bash
# Round 6 experiment 10 (via gpurun): the pass chain's kernels on their own -- C2 with serial iterations
# (--pipeline 0) under rocprofv3 --kernel-trace --stats, so every pass kernel's duration is its own, not
# the share it gets inside the other context's gather.
set -o pipefail
OUT=$1
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 -u bench.py --no-cpu --no-pmc \
    --no-legs --no-diag --pipeline 0 --steps 4 --warmup 1 > "$OUT/bench.log" 2>&1 || { tail -n 20 "$OUT/bench.log"; exit 1; }
find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
head -40 "$OUT/kernel_stats.csv" | cut -c1-100,200-400
