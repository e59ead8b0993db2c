#!/bin/bash
# A/B of library variants on the C3 bench: tools/ab_libs.sh OUT lib1 lib2 ... (default = the product library)
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for run in 1 2; do
  for lib in "$@"; do
    name=$(basename $lib .so)
    if [ "$lib" = default ]; then L=""; else L="SURF_HIP_LIB=$lib"; fi
    env $L timeout -k 10 200 python bench.py --no-cpu --steps 2 > "$OUT/${name}_$run.json" || exit 1
  done
done
for f in "$OUT"/*.json; do python3 -c "
import json; d=json.load(open('$f')); k=d['kernel_ms_profile_pass']; print('$f'.split('/')[-1], d['value'], d['ms_per_step'], 'ext', k['ms_extend'], 'con', k['ms_connect'], 'shade', k['ms_shade'], 'tail', k['ms_tail'])"; done
