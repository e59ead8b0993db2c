#!/bin/bash
# A/B: small-grid drain graph x wavefront-to-tail threshold on the C3 bench.
set -o pipefail
OUT=gpurun_out/${1:-ab_small}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
run() { name=$1; shift; env "$@" timeout -k 10 200 python bench.py --no-cpu --steps 2 $BARGS > "$OUT/$name.json" || exit 1; }
for r in 1 2; do
  BARGS="" run "sg0_default_$r" SURF_SMALL_GRAPH=0
  BARGS="" run "sg1_default_$r" SURF_SMALL_GRAPH=1
  BARGS="--tail 60000,0,16" run "sg1_t60k_$r" SURF_SMALL_GRAPH=1
  BARGS="--tail 30000,0,16" run "sg1_t30k_$r" SURF_SMALL_GRAPH=1
  BARGS="--tail 12000,0,16" run "sg1_t12k_$r" SURF_SMALL_GRAPH=1
done
for f in "$OUT"/*.json; do python3 -c "
import json; d=json.load(open('$f')); k=d['kernel_ms_profile_pass']; print('$f'.split('/')[-1], d['value'], d['ms_per_step'], 'ext', k['ms_extend'], 'con', k['ms_connect'], 'shade', k['ms_shade'], 'tail', k['ms_tail'], 'iters', d['iterations_per_render'], 'tailpaths', d['tail_paths_per_render'])"; done
