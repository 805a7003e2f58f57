#!/bin/bash
# r2: rehearsal of the multi-rank bench flow on a one-GPU box: 2 (and 4) ranks launched by
# bench.py --gpus N itself (torch.distributed.run), all on cuda:0, collectives over gloo; packet shards
set -o pipefail
O=gpurun_out/${EXPLORE_OUT:-rehearse_n2}; mkdir -p $O
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --share-gpu --steps 4 --warmup 1 --no-cpu --no-pmc \
    --json-out $O/n2.json > $O/n2.log 2>&1 || { tail -n 30 $O/n2.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/n2.json'));print('n2', d['n_gpus'], round(d['value']), round(d['ms_per_step'],1), d['estimates_per_step_per_gpu'], d['config']['parallelism'])"
timeout -k 10 300 python -u bench.py --gpus 4 --dist-backend gloo --share-gpu --steps 4 --warmup 1 --no-cpu --no-pmc \
    --shard-mode tiles --json-out $O/n4t.json > $O/n4t.log 2>&1 || { tail -n 30 $O/n4t.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/n4t.json'));print('n4 tiles', d['n_gpus'], round(d['value']), round(d['ms_per_step'],1), d['estimates_per_step_per_gpu'])"
