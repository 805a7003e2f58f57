#!/bin/bash
# Round 6 closing measurement (via gpurun), in three calls:
#   tests  -- smoke() and the whole GPU suite (full-size C1 image, C3 / C4 / C5 parity, class films);
#   bench  -- the default bench line (C2 16 steps: CPU leg, PMC roofline, counters at iterations 0 and 15,
#             C3 / C4 / C5 legs) and the driver-shaped line (--steps 20 --warmup 5);
#   prof   -- rocprofv3 kernel-trace / HBM passes of the same workload, the C-ABI boundary leg and the
#             multi-rank bench flow rehearsed with 1 / 2 / 4 ranks on the one GPU (gloo; film digests per N).
set -o pipefail
OUT=${1:-gpurun_out/r6/final}
PART=${2:-tests}
mkdir -p "$OUT"
( while sleep 60; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK' EXIT
export TMPDIR=/tmp
if [ "$PART" = tests ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 \
      || { tail -n 30 "$OUT/smoke.log"; exit 1; }
  tail -n 1 "$OUT/smoke.log"
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -s \
      > "$OUT/pytest_gpu.log" 2>&1 || { tail -n 40 "$OUT/pytest_gpu.log"; exit 1; }
  tail -n 1 "$OUT/pytest_gpu.log"
  grep -E "^C[1345]" "$OUT/pytest_gpu.log" | head -12
fi
if [ "$PART" = bench ]; then
  timeout -k 10 500 python -u bench.py --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1 \
      || { tail -n 30 "$OUT/bench.log"; exit 1; }
  tail -n 1 "$OUT/bench.log" | cut -c1-400
  timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 --json-out "$OUT/bench_driver.json" \
      > "$OUT/bench_driver.log" 2>&1 || { tail -n 30 "$OUT/bench_driver.log"; exit 1; }
  tail -n 1 "$OUT/bench_driver.log" | cut -c1-400
fi
if [ "$PART" = prof ]; then
  bash profiles/run_profiles.sh "$OUT" --steps 16 --warmup 1 --no-legs || { tail -n 20 "$OUT"/bench_*.log; exit 1; }
  cat "$OUT/summary.log"
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-legs --entry boundary --json-out "$OUT/bench_boundary.json" \
      > "$OUT/bench_boundary.log" 2>&1 || { tail -n 20 "$OUT/bench_boundary.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_boundary.json'));print('boundary', round(d['value']), round(d['ms_per_step'],1))"
  bash profiles/r6/rehearse.sh "$OUT/rehearse" || exit 1
fi
