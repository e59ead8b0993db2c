#!/bin/bash
# C5 (HBM-resident lattice BVH): k_extend / k_connect per render at 2/4/6/8
# trace waves per SIMD (launch bounds of the traversal kernels; builds
# lib/variants/s4t<N>.so, make -C surf-path-tracer_amd lib/variants/s4t<N>.so).
# One profiled C5 render per variant (HIP events per kernel).
# usage: tools/c5_waves_sweep.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/c5_waves}
mkdir -p "$OUT"
for n in 2 4 6 8; do
    lib=surf-path-tracer_amd/lib/variants/s4t$n.so
    [ "$n" = 2 ] && lib=surf-path-tracer_amd/lib/libsurf_hip.so
    SURF_HIP_LIB=$lib timeout -k 10 300 python bench.py --workload C5 --steps 1 --warmup 0 --no-cpu --profile-pass 1 \
        > "$OUT/t$n.json" 2> "$OUT/t$n.err" || { echo "variant t$n failed"; tail -5 "$OUT/t$n.err"; exit 1; }
    python3 -c "import json,sys; j=json.load(open('$OUT/t$n.json')); k=j['kernel_ms_profile_pass']; print('t$n', j['value'], 'Mrays/s', 'extend', k['ms_extend'], 'connect', k['ms_connect'], 'tail', k['ms_tail'])"
done
