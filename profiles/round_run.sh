#!/bin/bash
# One GPU-box pass for a round: gpu tests, the default bench line, then the rocprof passes.
# usage (from the repo root, via gpurun): profiles/round_run.sh TAG
set -o pipefail
TAG=${1:-rNN}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -n 30 "$OUT/pytest_gpu.log"; exit 1; }
tail -n 2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; cat "$OUT/smoke.log"; exit 1; }
timeout -k 10 600 bash profiles/run_profiles.sh "$OUT/prof" --steps 16 --warmup 2 || { echo profiles failed; exit 1; }
cat "$OUT/prof/summary.log"
timeout -k 10 400 python -u bench.py --json-out "$OUT/bench.json" \
    > "$OUT/bench.log" 2>&1 || { echo bench failed; tail -n 30 "$OUT/bench.log"; exit 1; }
cat "$OUT/bench.json"
