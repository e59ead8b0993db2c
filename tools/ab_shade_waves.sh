#!/bin/bash
# k_shade launch bound (waves per SIMD) A/B on C3: default build (4) vs lib/variants/s3t2.so / s5t2.so.
OUT=${1:-gpurun_out/ab_shade}
mkdir -p "$OUT"
for rep in 1 2; do
  for v in default s3t2 s5t2; do
    lib=surf-path-tracer_amd/lib/libsurf_hip.so; [ $v != default ] && lib=surf-path-tracer_amd/lib/variants/$v.so
    SURF_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --steps 2 > "$OUT/$v$rep.json" 2> "$OUT/$v$rep.err" || exit 1
    python3 -c "import json;j=json.load(open('$OUT/$v$rep.json'));k=j['kernel_ms_profile_pass'];print('$v$rep', j['value'], 'shade', k['ms_shade'], 'extend', k['ms_extend'], 'connect', k['ms_connect'], 'tail', k['ms_tail'])"
  done
done
