#!/bin/bash
# Round-3 measurement (via gpurun): smoke(), the default bench line (C2 16 iterations, CPU leg and the
# roofline's PMC passes included), then the rocprofv3 kernel-trace / HBM-counter passes of the same
# workload (profiles/run_profiles.sh).  usage: profiles/r3/final.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r3/final}
mkdir -p "$OUT"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 \
    || { tail -n 30 "$OUT/smoke.log"; exit 1; }
tail -n 1 "$OUT/smoke.log"
timeout -k 10 600 python -u bench.py --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1 \
    || { tail -n 30 "$OUT/bench.log"; exit 1; }
tail -n 1 "$OUT/bench.log"
bash profiles/run_profiles.sh "$OUT" --steps 16 --warmup 1 || { tail -n 20 "$OUT"/bench_*.log; exit 1; }
cat "$OUT/summary.log"
