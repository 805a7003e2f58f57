#!/bin/bash
# Round 4 measurement (via gpurun): smoke(), the whole GPU suite (C3, C4, C5 full-size parity included),
# the default bench line (C2: CPU leg, the roofline's PMC passes and the counter blocks at iterations 0
# and 15 included), the rocprofv3 kernel-trace / HBM passes of the same workload, the C-ABI boundary
# leg, C3 and C4 at N=1, and the multi-rank bench flow rehearsed with 2 / 4 ranks on the one GPU (gloo).
set -o pipefail
OUT=${1:-gpurun_out/r4/final}
PART=${2:-all}   # tests | bench | all (one gpurun call each for tests and bench keeps both inside 1200 s)
mkdir -p "$OUT"
( while sleep 60; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK' EXIT
export TMPDIR=/tmp
if [ "$PART" != bench ]; then
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 \
    || { tail -n 30 "$OUT/smoke.log"; exit 1; }
tail -n 1 "$OUT/smoke.log"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 1100 --timeout-method thread -s \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -n 40 "$OUT/pytest_gpu.log"; exit 1; }
tail -n 1 "$OUT/pytest_gpu.log"
grep -E "^C[345]" "$OUT/pytest_gpu.log" | head -12
fi
[ "$PART" = tests ] && exit 0
timeout -k 10 600 python -u bench.py --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1 \
    || { tail -n 30 "$OUT/bench.log"; exit 1; }
tail -n 1 "$OUT/bench.log" | cut -c1-600
bash profiles/run_profiles.sh "$OUT" --steps 16 --warmup 1 || { tail -n 20 "$OUT"/bench_*.log; exit 1; }
cat "$OUT/summary.log"
timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --entry boundary --json-out "$OUT/bench_boundary.json" \
    > "$OUT/bench_boundary.log" 2>&1 || { tail -n 20 "$OUT/bench_boundary.log"; exit 1; }
timeout -k 10 300 python -u bench.py --workload c3 --steps 1 --warmup 0 --no-cpu --no-pmc --json-out "$OUT/c3.json" \
    > "$OUT/c3.log" 2>&1 || { tail -n 20 "$OUT/c3.log"; exit 1; }
timeout -k 10 600 python -u bench.py --workload c4 --steps 1 --warmup 0 --no-cpu --no-pmc --no-diag \
    --json-out "$OUT/c4.json" > "$OUT/c4.log" 2>&1 || { tail -n 20 "$OUT/c4.log"; exit 1; }
EXPLORE_OUT=${OUT#gpurun_out/}/rehearse bash profiles/rehearse_n2.sh || exit 1
for f in bench bench_boundary c3 c4; do
  python3 -c "import json;d=json.load(open('$OUT/$f.json'));print('$f', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],1))"
done
