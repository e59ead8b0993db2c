#!/bin/bash
# Pool capacity A/B on C3: the default (~4 frames, 3.69 M paths) against 2x / 4x
# (fewer, larger wavefront phases); the drain hand-over kept at the default's
# 230 k paths.  usage: tools/ab_pool.sh OUT
OUT=${1:-gpurun_out/ab_pool}
mkdir -p "$OUT"
for rep in 1 2; do
  for pool in 0 7372800 14745600; do
    extra=""; [ $pool != 0 ] && extra="--pool $pool --tail 230400,0,16"
    timeout -k 10 300 python bench.py --no-cpu --steps 2 $extra > "$OUT/p${pool}_$rep.json" 2> "$OUT/p${pool}_$rep.err" || { tail -3 "$OUT/p${pool}_$rep.err"; exit 1; }
    python3 -c "import json;j=json.load(open('$OUT/p${pool}_$rep.json'));k=j['kernel_ms_profile_pass'];print('pool $pool', j['value'], 'iters', j['iterations_per_render'], 'extend', k['ms_extend'], 'shade', k['ms_shade'], 'connect', k['ms_connect'], 'sort', k['ms_sort'], 'tail', k['ms_tail'], 'tailpaths', k['tail_paths'])"
  done
done
