#!/bin/bash
# A/B: XCD-aware tiles (default build vs lib/variants/xcd0.so) x spatial ray keys, C3 and C5.
set -o pipefail
OUT=gpurun_out/${1:-ab_order}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
X0=surf-path-tracer_amd/lib/variants/xcd0.so
for run in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu --steps 2 > "$OUT/c3_xcd1_$run.json" || exit 1
  SURF_HIP_LIB=$X0 timeout -k 10 200 python bench.py --no-cpu --steps 2 > "$OUT/c3_xcd0_$run.json" || exit 1
done
timeout -k 10 200 python bench.py --workload C5 --no-cpu --steps 1 --warmup 0 > "$OUT/c5_xcd1_sp1.json" || exit 1
SURF_SPATIAL_KEYS=0 timeout -k 10 200 python bench.py --workload C5 --no-cpu --steps 1 --warmup 0 > "$OUT/c5_xcd1_sp0.json" || exit 1
SURF_HIP_LIB=$X0 timeout -k 10 200 python bench.py --workload C5 --no-cpu --steps 1 --warmup 0 > "$OUT/c5_xcd0_sp1.json" || exit 1
for f in "$OUT"/*.json; do python3 -c "
import json; d=json.load(open('$f')); k=d['kernel_ms_profile_pass']; print('$f'.split('/')[-1], d['value'], d['ms_per_step'], 'ext', k['ms_extend'], 'con', k['ms_connect'], 'shade', k['ms_shade'], 'tail', k['ms_tail'])"; done
