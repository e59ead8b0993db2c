#!/bin/bash
# Single-path segment latency + C3 bench per library variant: tools/ab_chain.sh OUT lib1 lib2 ... ("default" = product)
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for lib in "$@"; do
  name=$(basename $lib .so)
  if [ "$lib" = default ]; then L=""; else L="SURF_HIP_LIB=$lib"; fi
  env $L SURF_TAIL_ROWS=0 timeout -k 10 100 python tools/chain_probe2.py > "$OUT/chain_$name.txt" || exit 1
done
for run in 1 2; do
  for lib in "$@"; do
    name=$(basename $lib .so)
    if [ "$lib" = default ]; then L=""; else L="SURF_HIP_LIB=$lib"; fi
    env $L timeout -k 10 200 python bench.py --no-cpu --steps 2 > "$OUT/${name}_$run.json" || exit 1
  done
done
for f in "$OUT"/chain_*.txt; do echo "$f $(tail -1 $f)"; done
for f in "$OUT"/*.json; do python3 -c "
import json; d=json.load(open('$f')); k=d['kernel_ms_profile_pass']; print('$f'.split('/')[-1], d['value'], d['ms_per_step'], 'ext', k['ms_extend'], 'con', k['ms_connect'], 'shade', k['ms_shade'], 'tail', k['ms_tail'])"; done
