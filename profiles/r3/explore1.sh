#!/bin/bash
# Round 3 explore 1 (via gpurun): the tree-build beam key study (option 110: 0 centroid Morton, 1 start/end
# Morton) on the C2 bench, then the WorldBound sqrt-mode stakes, then the C4 test (exact-sum reference).
set -o pipefail
OUT=${1:-gpurun_out/r3/explore1}
mkdir -p "$OUT"
for bk in 0 1; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --beam-key $bk --json-out "$OUT/bk$bk.json" > "$OUT/bk$bk.log" 2>&1 \
      || { tail -n 20 "$OUT/bk$bk.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bk$bk.json'));print('beam key $bk', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]], 'staged/wave', round(d['beam_lines_staged_per_wave']), 'keep', round(d['bundle_keep_frac'],3), 'nodes/wave', round(d['node_visits_per_wave']), 'tests/q', round(d['prefilter_tests_per_queued_pair'],2))"
done
timeout -k 10 300 python -u profiles/r3/sqrt_mode.py 0,15 > "$OUT/sqrt_mode.log" 2>&1 || { tail -n 20 "$OUT/sqrt_mode.log"; exit 1; }
cat "$OUT/sqrt_mode.log"
timeout -k 10 700 python -u -m pytest tests/test_c4_gpu.py -m gpu -x -v -s --timeout 1100 --timeout-method thread \
    > "$OUT/pytest_c4.log" 2>&1 || { tail -n 40 "$OUT/pytest_c4.log"; exit 1; }
grep -E "C4|passed|failed" "$OUT/pytest_c4.log"
