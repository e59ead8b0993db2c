#!/bin/bash
# The drop-in 1-spp frame loop (examples/render_indoor, main.cpp:381-446) next to the batched bench.
set -o pipefail
OUT=gpurun_out/${1:-loop}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for r in 1 2; do
  timeout -k 10 120 surf-path-tracer_amd/build/render_indoor assets 1280 720 256 "$OUT/indoor_$r.png" > "$OUT/render_indoor_$r.txt" || exit 1
  tail -1 "$OUT/render_indoor_$r.txt"
done
timeout -k 10 200 python bench.py --no-cpu --steps 2 > "$OUT/c3.json" || exit 1
python3 -c "import json; d=json.load(open('$OUT/c3.json')); print('bench', d['value'], d['ms_per_step'])"
