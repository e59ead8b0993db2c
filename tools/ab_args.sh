#!/bin/bash
# A/B of bench.py argument sets on the C3 bench: tools/ab_args.sh OUT "args A" "args B" ... (two interleaved runs each)
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for run in 1 2; do
  i=0
  for a in "$@"; do
    i=$((i+1))
    timeout -k 10 200 python bench.py --no-cpu --steps 2 $a > "$OUT/v${i}_$run.json" || exit 1
  done
done
i=0; for a in "$@"; do i=$((i+1)); echo "v$i = $a"; done
for f in "$OUT"/*.json; do python3 -c "
import json; d=json.load(open('$f')); k=d['kernel_ms_profile_pass']; print('$f'.split('/')[-1], d['value'], d['ms_per_step'], 'ext', k['ms_extend'], 'con', k['ms_connect'], 'shade', k['ms_shade'], 'tail', k['ms_tail'])"; done
