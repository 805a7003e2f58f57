# quick GPU iteration with per-kernel stats: a short C2 bench under rocprofv3 --kernel-trace --stats
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/iterprof
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-diag "$@" > $OUT/bench.log 2>&1 || { tail -n 20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step','gather_kernel_ms')})"
python3 - $OUT <<'PY'
import csv, sys, os
rows = list(csv.DictReader(open(os.path.join(sys.argv[1], "t", "run_kernel_stats.csv"))))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    n = r["Name"].replace("bre::(anonymous namespace)::", "").replace("void ", "")[:60]
    print(f'{n:60s} calls {r["Calls"]:>4s} avg_ms {float(r["AverageNs"])/1e6:9.2f}')
PY
