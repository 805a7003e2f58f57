#!/bin/bash
# Round 4 run 30 (via gpurun): up to 1024 work roots -- S = 256 / 512 / 1024 at N = 1 and for an
# emulated rank 0 of 8 (C2), C3 at 256 / 512; parity tests at S = 1024 first.
set -o pipefail
OUT=${1:-gpurun_out/r4/run30}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_split_gpu.py \
    tests/test_gpu_parity.py tests/test_c2_production.py > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -n 60 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
run() { # name args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out "$OUT/$n.json" "$@" > "$OUT/$n.log" 2>&1 \
      || { tail -n 20 "$OUT/$n.log"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'gather', round(d['gather_kernel_ms'],2), [round(x,1) for x in d.get('gather_ms_per_step',[])][:4])"
}
for s in 256 512 1024; do
  run n1_s$s --split $s
  run r0of8_s$s --emulate-shard 0/8 --split $s
done
run c3_s256 --workload c3 --steps 1 --warmup 1
run c3_s512 --workload c3 --steps 1 --warmup 1 --split 512
