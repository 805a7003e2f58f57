#!/bin/bash
# r2: packet shards (every rank: whole camera pass + sort, then its range of the sorted packets):
# shard tests, then the strong-scaling emulation at N=8 / N=2 (C2, 16 iterations)
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore30}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_shard_gpu.py tests/test_camera_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -n 30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
c2() { n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || { tail -n 20 $O/c2_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c2_$n.json'));print('c2 $n', round(d['value']), 'ms/step', round(d['ms_per_step'],1), 'gather', round(d['gather_kernel_ms'],1), 'seg/step', round(d['estimates_per_step_per_gpu']))"
}
c2 n1 && c2 p0of8 --emulate-shard 0/8 && c2 p3of8 --emulate-shard 3/8 && c2 p7of8 --emulate-shard 7/8 \
 && c2 p5of8 --emulate-shard 5/8 && c2 p0of2 --emulate-shard 0/2 && c2 p1of2 --emulate-shard 1/2
