#!/bin/bash
# Round 3b run 1 (via gpurun): tight prefilter margins + mask-based scan (14 VALU per test) --
# the GPU suite without C4 (parity), the C2 bench with the new defaults, the same with round 2's
# margins (option 111 = 0) on the same box, then C3 one iteration.
set -o pipefail
OUT=${1:-gpurun_out/r3b/run1}
mkdir -p "$OUT"
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "not c4" \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -n 40 "$OUT/pytest_gpu.log"; exit 1; }
tail -n 2 "$OUT/pytest_gpu.log"
for m in 1 0; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --margin $m --json-out "$OUT/c2_m$m.json" > "$OUT/c2_m$m.log" 2>&1 \
      || { tail -n 20 "$OUT/c2_m$m.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c2_m$m.json'));print('margin $m value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]], 'q/est', round(d.get('queued_pairs_per_estimate',0)), 'tests/q', round(d.get('prefilter_tests_per_queued_pair',0),2), 'c/q', round(d.get('contributions_per_queued_pair',0),3), 'keep', round(d.get('bundle_keep_frac',0),3))"
done
timeout -k 10 300 python -u bench.py --workload c3 --steps 1 --warmup 0 --no-cpu --no-pmc --json-out "$OUT/c3.json" \
    > "$OUT/c3.log" 2>&1 || { tail -n 30 "$OUT/c3.log"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c3.json'));print('c3 value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1))"
