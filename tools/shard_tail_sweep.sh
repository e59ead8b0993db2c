#!/bin/bash
# 8-shard projection (tools/shard_probe.py 8) per drain hand-over threshold:
# the default (capacity/16) and lower ones that keep the wavefront on more of
# the short paths.  usage: tools/shard_tail_sweep.sh OUT
OUT=${1:-gpurun_out/shard_tail}
mkdir -p "$OUT"
for th in 0 60000 20000 8000; do
    if [ "$th" = 0 ]; then unset TAIL; else export TAIL="$th,0,16"; fi
    timeout -k 10 300 python tools/shard_probe.py 8 > "$OUT/th_$th.txt" 2>&1 || { tail -5 "$OUT/th_$th.txt"; exit 1; }
    echo "threshold $th: $(tail -1 $OUT/th_$th.txt)"
done
