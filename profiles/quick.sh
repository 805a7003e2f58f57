#!/bin/bash
# Quick GPU check of a kernel change (via gpurun): the production-path parity tests, then the C2
# bench without the CPU leg / PMC passes.  usage: profiles/quick.sh OUTDIR [extra bench args]
set -o pipefail
OUT=${1:-gpurun_out/quick}
shift || true
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_c2_production.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -n 30 "$OUT/pytest.log"; exit 1; }
tail -n 2 "$OUT/pytest.log"
timeout -k 10 400 python -u bench.py --no-cpu --no-pmc --json-out "$OUT/bench.json" "$@" > "$OUT/bench.log" 2>&1 \
    || { tail -n 20 "$OUT/bench.log"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('value', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
