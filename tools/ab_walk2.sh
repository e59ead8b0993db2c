#!/bin/bash
# A/B of the two-level wave walk (SURF_WALK2=1, default) against the one-level
# walk (SURF_WALK2=0) on one box: lone-path chain (pair drain), the timing
# build's per-segment split (coop drain), C3 drain and 8-shard slowest shard.
OUT=${1:-gpurun_out/ab_walk2}
mkdir -p "$OUT"
for w in 0 1 0 1; do
    SURF_WALK2=$w timeout -k 10 120 python tools/chain_probe.py > "$OUT/chain_$w.txt" 2>&1 || exit 1
    echo "walk2=$w chain: $(tail -1 $OUT/chain_$w.txt)"
done
for w in 0 1; do
    SURF_WALK2=$w SURF_HIP_LIB=surf-path-tracer_amd/lib/variants/timing.so SURF_DEBUG_TAIL=1 SURF_TAIL_PAIR=0 \
        timeout -k 10 120 python tools/chain_probe.py > "$OUT/timing_$w.txt" 2>&1 || exit 1
    echo "walk2=$w timing: $(grep 'coop cycles' $OUT/timing_$w.txt | tail -1)"
done
for w in 0 1; do
    SURF_WALK2=$w timeout -k 10 200 python tools/shard_breakdown.py 8 1 > "$OUT/shard_$w.txt" 2>&1 || exit 1
    echo "walk2=$w shard8/1: $(sed -n 2p $OUT/shard_$w.txt)"
done
