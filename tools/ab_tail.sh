#!/bin/bash
# A/B of drain engines x queue order on the C3 bench (profile pass: ms_tail).
set -o pipefail
OUT=gpurun_out/${1:-ab_tail}
mkdir -p "$OUT"
if [ "${2:-tests}" = tests ]; then
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
fi
for run in 1 2; do
  for cfg in "coop_sort:0:1" "coop_nosort:0:0" "rows_sort:1:1" "rows_nosort:1:0"; do
    IFS=: read name rows sort <<< "$cfg"
    SURF_TAIL_ROWS=$rows SURF_TAIL_SORT=$sort timeout -k 10 200 python bench.py --no-cpu --tail-coop 1000000 --steps 2 > "$OUT/${name}_$run.json" || exit 1
  done
  timeout -k 10 200 python bench.py --no-cpu --steps 2 > "$OUT/default_$run.json" || exit 1
done
for f in "$OUT"/*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); k=d['kernel_ms_profile_pass']; print('$f', d['value'], d['ms_per_step'], 'tail', k['ms_tail'], 'total', k['ms_total'])"; done
