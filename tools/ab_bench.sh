#!/bin/bash
# Same-box A/B of bench.py options on C3 (no -m gpu suite): one line per variant.
# usage: tools/ab_bench.sh OUT 'name:--opt v --opt v' ...
OUT=${1:-gpurun_out/abb}; shift
mkdir -p "$OUT"
for v in "$@"; do
  name=${v%%:*}; opts=${v#*:}
  timeout -k 10 240 python bench.py --no-cpu --steps 3 --warmup 1 $opts > "$OUT/$name.json" 2> "$OUT/$name.err" || exit 1
  python3 -c "import json;j=json.load(open('$OUT/$name.json'));k=j.get('kernel_ms_profile_pass');print('$name', j['value'], k['ms_tail'], k['tail_paths'])"
done
