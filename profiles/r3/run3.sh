#!/bin/bash
# Round 3 run 3 (via gpurun): the (start, end) tree order as the default -- the whole GPU suite
# (parity of the new tree), the C2 bench (tree key 1 vs 0 on one box), then the full-size C4 test.
set -o pipefail
OUT=${1:-gpurun_out/r3/run3}
mkdir -p "$OUT"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "not c4" \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -n 40 "$OUT/pytest_gpu.log"; exit 1; }
tail -n 2 "$OUT/pytest_gpu.log"
for bk in 1 0; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --beam-key $bk --json-out "$OUT/bk$bk.json" > "$OUT/bk$bk.log" 2>&1 \
      || { tail -n 20 "$OUT/bk$bk.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bk$bk.json'));print('tree key $bk', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]], 'staged/wave', round(d['beam_lines_staged_per_wave']), 'keep', round(d['bundle_keep_frac'],3), 'nodes/wave', round(d['node_visits_per_wave']), 'tests/q', round(d['prefilter_tests_per_queued_pair'],2), 'photon', round(d['photon_pass_ms'],2), 'build', round(d['bvh_build_ms'],2))"
done
timeout -k 10 700 python -u -m pytest tests/test_c4_gpu.py -m gpu -x -v -s --timeout 1100 --timeout-method thread \
    > "$OUT/pytest_c4.log" 2>&1 || { tail -n 40 "$OUT/pytest_c4.log"; exit 1; }
grep -E "C4|passed|failed" "$OUT/pytest_c4.log"
