set -o pipefail
mkdir -p gpurun_out/diag
for k in 3 0; do
timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu --kernel $k > gpurun_out/diag/k$k.log 2>&1 || { tail -n 20 gpurun_out/diag/k$k.log; exit 1; }
tail -n 1 gpurun_out/diag/k$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($k, {k: d[k] for k in ('gather_ms_iter0','node_visits_per_wave','leaf_visits_per_wave','beam_evals_per_wave','ccp_wave_evals_per_wave','prefilter_rejects_per_estimate','candidates_per_estimate','redo_items','max_stack_depth')})"
done
