#!/bin/bash
# quick GPU iteration: selected GPU tests (-k expr) + short C2 benches with the given arg sets
# usage (gpurun): profiles/iter2.sh OUT "pytest -k expr" "bench args 1" "bench args 2" ...
set -o pipefail
OUT=${1:-gpurun_out/iter2}; shift
K=$1; shift
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1 || { tail -n 40 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py ${STEPS:---steps 3 --warmup 1} --no-cpu $a > "$OUT/bench$i.log" 2>&1 || { tail -n 20 "$OUT/bench$i.log"; exit 1; }
  echo "[$a] $(grep '^{' "$OUT/bench$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: round(d.get(k),1) for k in ("value","ms_per_step","gather_kernel_ms","contributions_per_estimate","bundle_keep_frac","bvh_build_ms","photon_pass_ms") if d.get(k) is not None})')"
done
