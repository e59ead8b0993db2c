#!/bin/bash
# A/B of an environment knob on the C3 bench: tools/ab_env.sh OUT VAR v1 v2 ... (two interleaved runs each)
set -o pipefail
OUT=gpurun_out/$1; VAR=$2; shift 2
mkdir -p "$OUT"
for run in 1 2; do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 200 python bench.py --no-cpu --steps 2 > "$OUT/${VAR}_${v}_$run.json" || exit 1
  done
done
for f in "$OUT"/*.json; do python3 -c "
import json; d=json.load(open('$f')); k=d['kernel_ms_profile_pass']; print('$f'.split('/')[-1], d['value'], d['ms_per_step'], 'ext', k['ms_extend'], 'con', k['ms_connect'], 'shade', k['ms_shade'], 'tail', k['ms_tail'])"; done
