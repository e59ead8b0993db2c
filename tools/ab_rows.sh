#!/bin/bash
# A/B of the drain engines on the C3 bench: four-rows tail vs one path per wave.
set -o pipefail
OUT=gpurun_out/${1:-ab_rows}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
for run in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu > "$OUT/rows60k_$run.json" || exit 1
  timeout -k 10 200 python bench.py --no-cpu --tail-coop 1000000 > "$OUT/rowsall_$run.json" || exit 1
  SURF_TAIL_ROWS=0 timeout -k 10 200 python bench.py --no-cpu > "$OUT/coop_$run.json" || exit 1
done
for f in "$OUT"/*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); k=d['kernel_ms_profile_pass']; print('$f', d['value'], d['ms_per_step'], 'tail', k['ms_tail'], 'total', k['ms_total'])"; done
