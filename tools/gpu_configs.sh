#!/bin/bash
# BASELINE configs on one GPU: C4 / C2 / C5 bench lines, C3 streams longer than
# 256 frames (window check), the drop-in frame loop, C4 shard projection.
set -o pipefail
OUT=gpurun_out/${1:-configs}
mkdir -p "$OUT"
timeout -k 10 240 python bench.py --workload C4 --steps 1 --warmup 1 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" || { echo c4 failed; tail "$OUT/bench_c4.err"; exit 1; }
timeout -k 10 200 python bench.py --workload C2 --steps 3 --warmup 1 > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || { echo c2 failed; exit 1; }
timeout -k 10 240 python bench.py --workload C5 --steps 2 --warmup 1 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" || { echo c5 failed; tail "$OUT/bench_c5.err"; exit 1; }
for spp in 320 1024; do
  timeout -k 10 200 python bench.py --spp $spp --steps 1 --warmup 1 --no-cpu > "$OUT/bench_c3_spp$spp.json" || { echo spp failed; exit 1; }
done
timeout -k 10 120 surf-path-tracer_amd/build/render_indoor assets 1280 720 256 "$OUT/indoor_256.png" > "$OUT/render_indoor_256.txt" || { echo render_indoor failed; exit 1; }
tail -1 "$OUT/render_indoor_256.txt"
W=1920 H=1080 F=1024 timeout -k 10 300 python tools/shard_probe.py 1,8 > "$OUT/shards_c4.txt" || { echo shard probe failed; exit 1; }
F=256 timeout -k 10 200 python tools/shard_probe.py 8 > "$OUT/shards_c3.txt" || { echo shard probe c3 failed; exit 1; }
grep slowest "$OUT"/shards_*.txt
for f in "$OUT"/bench_*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], (d.get('kernel_ms_profile_pass') or {}).get('ms_tail'), (d.get('cpu_baseline') or {}).get('value'), (d.get('parity') or {}).get('bitexact'))"; done
