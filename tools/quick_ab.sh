#!/bin/bash
# Quick check of a traversal change: -m gpu tests, single-path segment latency, two C3 bench runs.
set -o pipefail
OUT=gpurun_out/${1:-quick}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
SURF_TAIL_ROWS=0 timeout -k 10 100 python tools/chain_probe2.py > "$OUT/chain.txt" || exit 1
cat "$OUT/chain.txt"
for run in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu --steps 2 > "$OUT/c3_$run.json" || exit 1
done
for f in "$OUT"/c3_*.json; do python3 -c "
import json; d=json.load(open('$f')); k=d['kernel_ms_profile_pass']; print('$f'.split('/')[-1], d['value'], d['ms_per_step'], 'ext', k['ms_extend'], 'con', k['ms_connect'], 'shade', k['ms_shade'], 'tail', k['ms_tail'])"; done
