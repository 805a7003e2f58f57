#!/bin/bash
# r2: two-context pipelining (iteration k+1's photon pass / build / camera pass overlap iteration k's
# gather) vs one context; N=1 and an emulated 1/8 packet shard
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore34}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -n 30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
c2() { n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || { tail -n 20 $O/c2_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c2_$n.json'));print('c2 $n', round(d['value']), 'ms/step', round(d['ms_per_step'],1), 'gather', round(d['gather_kernel_ms'],1))"
}
c2 pipe1 && c2 pipe0 --pipeline 0 && c2 p0of8pipe1 --emulate-shard 0/8 && c2 p0of8pipe0 --emulate-shard 0/8 --pipeline 0
