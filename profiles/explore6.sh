#!/bin/bash
set -o pipefail
O=gpurun_out/explore6; mkdir -p $O
timeout -k 10 200 python -u profiles/depth_split.py c2 0 > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 1; }
timeout -k 10 300 python -u profiles/depth_split.py c3 0 > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
grep -v "^{" $O/c2.log $O/c3.log
