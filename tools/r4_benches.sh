#!/bin/bash
# Round-4 bench lines (C3 default + C2/C4/C5), the N = 2 bench path rehearsed on one GPU
# (two ranks on device 0, gloo gather, assembled frame checked against the oracle), and the
# 8-shard projections of C3 and C4.  usage: tools/r4_benches.sh OUT
OUT=${1:-gpurun_out/r4_bench}
mkdir -p "$OUT"
timeout -k 10 400 python bench.py > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" || { tail -5 "$OUT/bench_c3.err"; exit 1; }
echo "C3 $(python3 -c "import json;j=json.load(open('$OUT/bench_c3.json'));print(j['value'], j['parity']['bitexact'], j['gpu_vs_cpu'], j['roofline']['frac'])")"
for wl in C2 C4 C5; do
    timeout -k 10 500 python bench.py --workload $wl > "$OUT/bench_${wl,,}.json" 2> "$OUT/bench_${wl,,}.err" || { tail -5 "$OUT/bench_${wl,,}.err"; exit 1; }
    echo "$wl $(python3 -c "import json;j=json.load(open('$OUT/bench_${wl,,}.json'));print(j['value'], j['parity']['bitexact'], j['gpu_vs_cpu'], j['roofline']['frac'])")"
done
SURF_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 > "$OUT/dist_n2.json" 2> "$OUT/dist_n2.err" || { tail -5 "$OUT/dist_n2.err"; exit 1; }
echo "N2 $(tail -1 $OUT/dist_n2.json | python3 -c "import json,sys;j=json.loads(sys.stdin.read());print(j['value'], j['parity'], j['roofline'])")"
timeout -k 10 300 python tools/shard_probe.py 8 > "$OUT/shards8_c3.txt" 2>&1 || exit 1
tail -1 "$OUT/shards8_c3.txt"
W=1920 H=1080 F=1024 timeout -k 10 600 python tools/shard_probe.py 8 > "$OUT/shards8_c4.txt" 2>&1 || exit 1
tail -1 "$OUT/shards8_c4.txt"
