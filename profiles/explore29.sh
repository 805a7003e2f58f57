#!/bin/bash
# r2: per-packet work of one emulated rank's share (counters pass) vs the whole film: N=1, 0/8, 0/8 block 4
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-explore29}; mkdir -p $O
c2() { n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --steps 4 --json-out $O/c2_$n.json "$@" > $O/c2_$n.log 2>&1 || { tail -n 20 $O/c2_$n.log; return 1; }
  python3 -c "
import json;d=json.load(open('$O/c2_$n.json'))
print('c2 $n', round(d['value']), 'gather', round(d['gather_kernel_ms'],1), 'it0', round(d['gather_ms_iter0'],1), 'segs', round(d['estimates_per_step_per_gpu']))
print('   nodes/w', round(d['node_visits_per_wave'],1), 'leaves/w', round(d['leaf_visits_per_wave'],1), 'staged/w', round(d['beam_lines_staged_per_wave']), 'batches/w', round(d['exact_batches_per_wave'],1), 'keep', round(d['bundle_keep_frac'],3), 'cand/est', round(d['candidates_per_estimate']), 'contrib/est', round(d['contributions_per_estimate']))"
}
c2 n1 && c2 r0of8 --emulate-shard 0/8 && c2 r0of8b4 --emulate-shard 0/8 --shard-block 4 && c2 r0of8s64 --emulate-shard 0/8 --split 64
