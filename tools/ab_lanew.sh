#!/bin/bash
# A/B of the lane traversal over two-level records (SURF_LANEW=1) against the
# one-level lane walk (SURF_LANEW=0) on C5 and C3: one profiled render each.
OUT=${1:-gpurun_out/ab_lanew}
mkdir -p "$OUT"
for wl in C5 C3; do
    for w in 0 1; do
        SURF_LANEW=$w timeout -k 10 300 python bench.py --workload $wl --steps 1 --warmup 0 --no-cpu --profile-pass 1 \
            > "$OUT/${wl}_$w.json" 2> "$OUT/${wl}_$w.err" || { tail -5 "$OUT/${wl}_$w.err"; exit 1; }
        python3 -c "import json; j=json.load(open('$OUT/${wl}_$w.json')); k=j['kernel_ms_profile_pass']; print('$wl lanew=$w', j['value'], 'Mrays/s', 'extend', k['ms_extend'], 'connect', k['ms_connect'], 'tail', k['ms_tail'], 'frac', j['roofline']['frac'])"
    done
done
