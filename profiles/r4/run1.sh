#!/bin/bash
# Round 4 run 1 (via gpurun): the new GPU tests (device primitive check, transposed-scan queue, RCCL
# world-1 collectives, C3 / C5 full-size parity), then a C2 baseline line of the round-3 kernel.
set -o pipefail
OUT=${1:-gpurun_out/r4/run1}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread \
    tests/test_device_check_gpu.py tests/test_rccl_gpu.py tests/test_c3_c5_gpu.py \
    "tests/test_gpu_parity.py::test_transposed_scan_skips_packet_rejected_parallel_beams" \
    > "$OUT/pytest_new.log" 2>&1 || { echo "pytest failed"; tail -n 40 "$OUT/pytest_new.log"; exit 1; }
tail -n 3 "$OUT/pytest_new.log"
timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --json-out "$OUT/base.json" > "$OUT/base.log" 2>&1 \
    || { echo bench failed; tail -n 30 "$OUT/base.log"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/base.json'));print('base value', round(d['value']), 'ms', round(d['ms_per_step'],1))"
