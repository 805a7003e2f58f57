#!/bin/bash
# Per-kernel gather time under the timing-only debug modes (0 full, 1 traversal only, 2 no
# distance work, 3 no exact closest points): where kernel 3 / kernel 4 time goes.
# usage (gpurun, repo root): profiles/dbgsplit.sh OUTDIR [extra bench args]
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/dbg}; shift
mkdir -p "$OUT"
for m in 0 1 2 3; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/m$m" -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu --no-diag --debug-mode $m "$@" > "$OUT/m$m.log" 2>&1 || { tail -n 20 "$OUT/m$m.log"; exit 1; }
  python3 - "$OUT/m$m/run_kernel_stats.csv" $m <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    n = r["Name"]
    if "gather" in n or "k_reduce" in n or "k_chunk" in n:
        short = n.replace("void ", "").replace("bre::(anonymous namespace)::", "").split("(")[0]
        out.append(f'{short}: {float(r["AverageNs"])/1e6:.1f} ms x{r["Calls"]}')
print("mode", sys.argv[2], "|", "; ".join(out))
PY
done
