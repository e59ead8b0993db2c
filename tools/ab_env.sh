#!/bin/bash
# A/B of library knobs on C3 (environment variables read by libsurf_hip):
# the -m gpu suite with the defaults, then one bench line per variant.
# usage: tools/ab_env.sh OUT [variant ...]   variant = name:ENV=V,ENV=V
OUT=${1:-gpurun_out/ab}; shift
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  ( IFS=,; for e in $envs; do export "$e"; done
    timeout -k 10 240 python bench.py --no-cpu --steps 3 --warmup 1 > "$OUT/$name.json" 2> "$OUT/$name.err" ) || exit 1
  python3 -c "import json;j=json.load(open('$OUT/$name.json'));print('$name', j['value'], j.get('kernel_ms_profile_pass'))"
done
