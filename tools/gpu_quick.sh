#!/bin/bash
# Quick GPU check of a drain change: drain parity tests, lone chain, 8-shard
# breakdown of shard 1, one profiled C3 render.  usage: tools/gpu_quick.sh OUT
OUT=${1:-gpurun_out/quick}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "drain_policies or general_tlas or render_64 or c1_256 or closest_hit or any_hit" > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/chain_probe.py > "$OUT/chain.txt" 2>&1 || exit 1
tail -1 "$OUT/chain.txt"
timeout -k 10 200 python tools/shard_breakdown.py 8 1 > "$OUT/shard.txt" 2>&1 || exit 1
sed -n 2,3p "$OUT/shard.txt"
timeout -k 10 300 python bench.py --no-cpu > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
python3 -c "import json;j=json.load(open('$OUT/bench.json'));print(j['value'], j['kernel_ms_profile_pass'])"
