#!/bin/bash
# Round 6 experiment 2 (via gpurun): the one-wave pass chain (bre_slot.hip) -- its unit tests, the GPU
# suite, then the pipelined C2 bench with the new chain (default) against option 119 = 0 (rocPRIM /
# hipMemset on the chain), each with a kernel trace for the gaps between the gathers.
# usage: bash profiles/r6/e2.sh OUT [tests|bench|all]
set -o pipefail
OUT=$1; PART=${2:-all}
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 60; do echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK' EXIT
if [ "$PART" != bench ]; then
  timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_slot_gpu.py \
      tests/test_work_roots_gpu.py tests/test_pass_stream_gpu.py > "$OUT/pytest_new.log" 2>&1 \
      || { echo "new tests failed"; tail -n 40 "$OUT/pytest_new.log"; exit 1; }
  tail -n 1 "$OUT/pytest_new.log"
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1 || { echo "gpu suite failed"; tail -n 40 "$OUT/pytest_gpu.log"; exit 1; }
  tail -n 1 "$OUT/pytest_gpu.log"
fi
if [ "$PART" != tests ]; then
  run() { # name args...
    n=$1; shift
    timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-legs --no-diag --json-out "$OUT/$n.json" "$@" \
        > "$OUT/$n.log" 2>&1 || { tail -n 20 "$OUT/$n.log"; exit 1; }
    python3 - "$OUT/$n.json" "$n" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], round(d["value"]), "ms/step", round(d["ms_per_step"], 3), "gather", round(d["gather_kernel_ms"], 3),
      "gap", round(d["ms_per_step"] - d["gather_kernel_ms"], 3), "digest", (d.get("film_digest") or {}).get("sha256"))
PY
  }
  trace() { # name args...
    n=$1; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr_$n" -o run -- \
        python3 bench.py --no-cpu --no-pmc --no-legs --no-diag "$@" > "$OUT/tr_$n.log" 2>&1 || { tail -n 20 "$OUT/tr_$n.log"; exit 1; }
    python3 profiles/r6/gap.py "$OUT/tr_$n/run_kernel_trace.csv" "$n"
  }
  for r in a b; do
    run slot_$r
    run rocprim_$r --slot-passes 0
  done
  run slot_emul8 --emulate-shard 0/8
  run rocprim_emul8 --emulate-shard 0/8 --slot-passes 0
  trace slot
  trace rocprim --slot-passes 0
fi
