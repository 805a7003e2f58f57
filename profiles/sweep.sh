set -e
mkdir -p gpurun_out/sweep8
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_camera_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sweep8/pytest.log 2>&1
for cfg in "--workload synthetic" "--workload c2"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu $cfg --json-out gpurun_out/sweep8/$tag.json > gpurun_out/sweep8/$tag.log 2>&1
  echo "$cfg done"
done
