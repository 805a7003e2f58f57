#!/bin/bash
# Round 4 run 23 (via gpurun): kernel trace of an emulated 1/8 rank (C2, rank 0 of 8, passes serialised)
# and of N = 1 the same way, to see what a rank's iteration spends beyond 1/8 of the gather.
set -o pipefail
OUT=${1:-gpurun_out/r4/run23}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r0of8" -o run -- \
    python3 bench.py --emulate-shard 0/8 --pipeline 0 --steps 16 --warmup 1 --no-cpu --no-pmc --no-diag > "$OUT/r0of8.log" 2>&1 \
    || { tail -n 20 "$OUT/r0of8.log"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/n1" -o run -- \
    python3 bench.py --pipeline 0 --steps 16 --warmup 1 --no-cpu --no-pmc --no-diag > "$OUT/n1.log" 2>&1 \
    || { tail -n 20 "$OUT/n1.log"; exit 1; }
for x in r0of8 n1; do
  echo "== $x"
  python3 - "$OUT/$x/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:16]:
    print("%9.2f ms %5s calls  avg %9.1f us  %s" % (float(r['TotalDurationNs']) / 1e6, r['Calls'], float(r['AverageNs']) / 1e3, r['Name'][:90]))
PY
done
