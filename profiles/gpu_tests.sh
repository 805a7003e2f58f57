#!/bin/bash
# GPU test pass only (via gpurun): profiles/gpu_tests.sh OUTDIR [pytest -k expr]
set -o pipefail
OUT=${1:-gpurun_out/tests}
mkdir -p "$OUT"
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > "$OUT/pytest_gpu.log" 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
fi
rc=$?
tail -n 40 "$OUT/pytest_gpu.log"
exit $rc
