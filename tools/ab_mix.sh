#!/bin/bash
# Same-box A/B mixing environment knobs and bench.py options on any workload:
# usage: tools/ab_mix.sh OUT 'name|ENV=V,ENV=V|--opt v --opt v' ...
OUT=${1:-gpurun_out/abm}; shift
mkdir -p "$OUT"
for v in "$@"; do
  IFS='|' read -r name envs opts <<< "$v"
  ( IFS=,; for e in $envs; do [ -n "$e" ] && export "$e"; done; unset IFS
    timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 $opts > "$OUT/$name.json" 2> "$OUT/$name.err" ) || exit 1
  python3 -c "import json;j=json.load(open('$OUT/$name.json'));k=j.get('kernel_ms_profile_pass');print('$name', j['value'], 'ext', k['ms_extend'], 'tail', k['ms_tail'], k['tail_paths'], 'it', j['iterations_per_render'])"
done
