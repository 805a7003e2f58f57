#!/bin/bash
# GPU tests + a short C2 bench for each kernel choice given (via gpurun): profiles/cmp.sh OUT "args1" "args2" ...
set -o pipefail
OUT=${1:-gpurun_out/cmp}; shift
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -n 40 "$OUT/pytest_gpu.log"; exit 1; }
tail -n 1 "$OUT/pytest_gpu.log"
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu $a > "$OUT/bench$i.log" 2>&1 || { tail -n 20 "$OUT/bench$i.log"; exit 1; }
  echo "[$a] $(grep '^{' "$OUT/bench$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ("value","ms_per_step","gather_kernel_ms","candidates_per_estimate","contributions_per_estimate")})')"
done
