set -o pipefail
mkdir -p gpurun_out/k5
timeout -k 10 600 python -u -m pytest tests/test_chunk_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/k5/pytest.log 2>&1; rc=$?
tail -n 25 gpurun_out/k5/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --kernel 5 --steps 3 --warmup 1 --no-cpu > gpurun_out/k5/bench5.log 2>&1 || { tail -n 20 gpurun_out/k5/bench5.log; exit 1; }
tail -n 1 gpurun_out/k5/bench5.log
