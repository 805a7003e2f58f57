#!/bin/bash
# r2: work roots sorted by size (largest first) + block map 3 (all packets on the largest subtree first:
# LPT, a tail of small waves) vs the rotated map 1; N=1 and emulated packet shards of N=8
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore32}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_c2_production.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -n 30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
c2() { n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || { tail -n 20 $O/c2_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c2_$n.json'));print('c2 $n', round(d['value']), 'ms/step', round(d['ms_per_step'],1), 'gather', round(d['gather_kernel_ms'],1), 'seg/step', round(d['estimates_per_step_per_gpu']))"
}
c3() { n=$1; shift
  timeout -k 10 300 python -u bench.py --workload c3 --steps 1 --warmup 0 --no-cpu --no-pmc --no-diag --json-out $O/c3_$n.json "$@" > $O/c3_$n.log 2>&1 || { tail -n 20 $O/c3_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c3_$n.json'));print('c3 $n', round(d['value']), round(d['gather_kernel_ms'],1))"
}
c2 m1 --block-map 1 && c2 m3 --block-map 3 && c2 p0of8m1 --emulate-shard 0/8 --block-map 1 && c2 p0of8m3 --emulate-shard 0/8 --block-map 3 \
 && c2 p5of8m3 --emulate-shard 5/8 --block-map 3 && c3 m1 --block-map 1 && c3 m3 --block-map 3
