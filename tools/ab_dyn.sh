#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-ab_dyn}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
SURF_EXTEND_DYN=1 timeout -k 10 200 python bench.py --workload C5 --no-cpu --steps 1 --warmup 0 > "$OUT/c5_dyn1.json" || exit 1
SURF_EXTEND_DYN=1 SURF_GRID_DYN=4 timeout -k 10 200 python bench.py --workload C5 --no-cpu --steps 1 --warmup 0 > "$OUT/c5_dyn1_g4.json" || exit 1
SURF_EXTEND_DYN=1 timeout -k 10 200 python bench.py --no-cpu --steps 2 > "$OUT/c3_dyn1.json" || exit 1
SURF_EXTEND_DYN=0 timeout -k 10 200 python bench.py --no-cpu --steps 2 > "$OUT/c3_dyn0.json" || exit 1
for f in "$OUT"/*.json; do python3 -c "
import json; d=json.load(open('$f')); k=d['kernel_ms_profile_pass']; print('$f'.split('/')[-1], d['value'], d['ms_per_step'], 'ext', k['ms_extend'], 'con', k['ms_connect'], 'shade', k['ms_shade'], 'tail', k['ms_tail'])"; done
