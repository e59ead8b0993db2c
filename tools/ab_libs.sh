#!/bin/bash
# Same-box A/B of two library builds (SURF_HIP_LIB): lone chain, 8-shard shard 1,
# one profiled C3 render each, interleaved A B A B.
# usage: tools/ab_libs.sh OUT LIB_A LIB_B
OUT=${1:-gpurun_out/ab}; A=$2; B=$3
mkdir -p "$OUT"
for rep in 1 2; do
  for tag in A B; do
    lib=$A; [ $tag = B ] && lib=$B
    SURF_HIP_LIB=$lib timeout -k 10 120 python tools/chain_probe.py > "$OUT/chain_${tag}$rep.txt" 2>&1 || exit 1
    SURF_HIP_LIB=$lib timeout -k 10 200 python tools/shard_breakdown.py 8 1 > "$OUT/shard_${tag}$rep.txt" 2>&1 || exit 1
    SURF_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --steps 2 > "$OUT/bench_${tag}$rep.json" 2> "$OUT/bench_${tag}$rep.err" || exit 1
    echo "$tag$rep chain $(tail -1 $OUT/chain_${tag}$rep.txt | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["us_per_segment"])') shard $(sed -n 3p $OUT/shard_${tag}$rep.txt | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["wall_ms"])') bench $(python3 -c "import json;j=json.load(open('$OUT/bench_${tag}$rep.json'));k=j['kernel_ms_profile_pass'];print(j['value'], 'tail', k['ms_tail'])")"
  done
done
