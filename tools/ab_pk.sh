#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-ab_pk}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for r in 1 2; do
  SURF_CONNECT_PACKET=0 timeout -k 10 200 python bench.py --no-cpu --steps 2 > "$OUT/pk0_$r.json" || exit 1
  SURF_CONNECT_PACKET=1 timeout -k 10 200 python bench.py --no-cpu --steps 2 > "$OUT/pk1_$r.json" || exit 1
done
SURF_CONNECT_PACKET=1 timeout -k 10 200 python bench.py --workload C5 --no-cpu --steps 1 --warmup 0 > "$OUT/c5_pk1.json" || exit 1
for f in "$OUT"/*.json; do python3 -c "
import json; d=json.load(open('$f')); k=d['kernel_ms_profile_pass']; print('$f'.split('/')[-1], d['value'], d['ms_per_step'], 'ext', k['ms_extend'], 'con', k['ms_connect'], 'shade', k['ms_shade'], 'tail', k['ms_tail'])"; done
