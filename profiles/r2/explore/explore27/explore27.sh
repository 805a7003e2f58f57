#!/bin/bash
# r2: the transposed-scan bit-identity test, and the segment sort key re-checked on the final kernel
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore27}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k transposed --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -n 30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
c2() { n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --no-diag --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || { tail -n 20 $O/c2_$n.log; return 1; }
  python3 -c "import json;d=json.load(open('$O/c2_$n.json'));print('c2 $n', round(d['value']), round(d['gather_kernel_ms'],1), [round(x) for x in d['gather_ms_per_step'][::3]])"
}
c2 key1 && c2 key0 --sort-key 0
