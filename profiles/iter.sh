# quick GPU iteration: parity tests + a short C2 bench (gpurun from the repo root)
set -o pipefail
OUT=gpurun_out/iter
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_camera_gpu.py tests/test_chunk_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -n 40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu "$@" > $OUT/bench.log 2>&1 || { tail -n 20 $OUT/bench.log; exit 1; }
tail -n 1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step','gather_kernel_ms','gather_ms_iter0','candidates_per_estimate','contributions_per_estimate','ccp_wave_evals_per_wave','redo_items')})"
