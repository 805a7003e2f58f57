set -o pipefail
mkdir -p gpurun_out/k0sort
timeout -k 10 300 python -u -m pytest tests/test_camera_gpu.py -x -q --timeout 200 --timeout-method thread -k "sort or render" > gpurun_out/k0sort/pytest.log 2>&1 || { tail -n 30 gpurun_out/k0sort/pytest.log; exit 1; }
tail -n 2 gpurun_out/k0sort/pytest.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/k0sort/bench_sort1.log 2>&1 || { tail -n 20 gpurun_out/k0sort/bench_sort1.log; exit 1; }
tail -n 1 gpurun_out/k0sort/bench_sort1.log | cut -c1-700
