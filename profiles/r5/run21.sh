#!/bin/bash
# Round 5 run 21 (via gpurun): the pass-rate-adaptive transposed-scan threshold (tscan - tslope * rho,
# option 118): parity, sums bit for bit against the fixed threshold (tslope 0), then C2 / C3 sweeps.
set -o pipefail
OUT=${1:-gpurun_out/r5/run21}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
    tests/test_c2_production.py tests/test_gpu_parity.py tests/test_prefilter_options_gpu.py \
    tests/test_film_determinism_gpu.py > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -n 40 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-legs --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));g=d['gather_ms_per_step'];print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'g', [round(x,1) for x in g])"
}
run c2_s15
run c2_s0 --tslope 0
run c2_s10 --tslope 10
run c2_s20 --tslope 20
run c2_t7s20 --tscan 7 --tslope 20
run c2_t5s10 --tscan 5 --tslope 10
for a in "--tslope 15" "--tslope 0" "--tslope 10" "--tslope 20" "--tscan 7 --tslope 20" "--tscan 5 --tslope 10"; do
  run "c3_$(echo $a | tr -d ' -')" --workload c3 --steps 1 --warmup 1 $a
done
run c2_s15_b
run c2_s0_b --tslope 0
