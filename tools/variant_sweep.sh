#!/bin/bash
# Bench each occupancy variant (surf-path-tracer_amd/lib/variants/*.so) on the GPU box.
set -e
OUT=${1:-gpurun_out/variants}
mkdir -p "$OUT"
for v in surf-path-tracer_amd/lib/variants/*.so; do
    n=$(basename "$v" .so)
    SURF_HIP_LIB="$PWD/$v" timeout -k 10 200 python3 bench.py --no-cpu --steps 16 > "$OUT/$n.json" 2> "$OUT/$n.err"
    echo "$n $(python3 -c "import json;d=json.load(open('$OUT/$n.json'));print(d['value'], d['kernel_ms_profile_pass'])")"
done
