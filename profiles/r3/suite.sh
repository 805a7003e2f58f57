#!/bin/bash
# Round-3 GPU pass (via gpurun): the GPU suite without C4, the C2 bench (camera entry, then the
# C-ABI boundary entry), then the full-size C4 test.  usage: profiles/r3/suite.sh OUTDIR [skip_c4]
set -o pipefail
OUT=${1:-gpurun_out/r3}
mkdir -p "$OUT"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "not c4" \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -n 40 "$OUT/pytest_gpu.log"; exit 1; }
tail -n 2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --json-out "$OUT/bench_camera.json" > "$OUT/bench_camera.log" 2>&1 \
    || { tail -n 20 "$OUT/bench_camera.log"; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --entry boundary --json-out "$OUT/bench_boundary.json" \
    > "$OUT/bench_boundary.log" 2>&1 || { tail -n 20 "$OUT/bench_boundary.log"; exit 1; }
for f in camera boundary; do
  python3 -c "import json;d=json.load(open('$OUT/bench_$f.json'));print('$f', 'value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]], 'q/est', round(d.get('queued_pairs_per_estimate',0)), 'tests/q', round(d.get('prefilter_tests_per_queued_pair',0),2))"
done
for it in ${DEPTH_KEYS_ITERS:-}; do
  timeout -k 10 200 python -u profiles/r3/depth_keys.py c2 $it 1,2,3 > "$OUT/depth_keys_c2_$it.log" 2>&1 \
      || { tail -n 20 "$OUT/depth_keys_c2_$it.log"; exit 1; }
  grep -v '^{' "$OUT/depth_keys_c2_$it.log" | python3 -c "
import sys, json
for ln in sys.stdin:
    name, js = ln.split(' ', 1); d = json.loads(js)
    print('it $it', name, 'k', d['key'], 'ms', round(d['gather_ms'], 1), 'kept/pk', round(d['kept_per_packet']), 'tests/q', round(d['tests_per_queued'], 2))"
done
[ "$2" = "skip_c4" ] && exit 0
timeout -k 10 700 python -u -m pytest tests/test_c4_gpu.py -m gpu -x -v -s --timeout 1100 --timeout-method thread \
    > "$OUT/pytest_c4.log" 2>&1 || { tail -n 40 "$OUT/pytest_c4.log"; exit 1; }
tail -n 6 "$OUT/pytest_c4.log"
