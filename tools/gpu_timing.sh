#!/bin/bash
# Lone-path segment timing breakdown (SURF_SEG_TIMING build, k_tail_coop): cycles per
# segment in extend / shade / connect and the extension's prologue / BLAS-walk split.
# usage: tools/gpu_timing.sh OUT
OUT=${1:-gpurun_out/timing}
mkdir -p "$OUT"
SURF_HIP_LIB=surf-path-tracer_amd/lib/variants/timing.so SURF_DEBUG_TAIL=1 SURF_TAIL_PAIR=0  \
    timeout -k 10 120 python tools/chain_probe.py > "$OUT/chain_timing.txt" 2>&1
rc=$?
grep -E "cycles|us_per" "$OUT/chain_timing.txt" | tail -4
exit $rc
