#!/bin/bash
# End-of-round check on one GPU: the whole -m gpu suite, smoke, the bench lines
# (C3/C2/C4/C5 + the N = 2 rehearsal), the 8-shard projection and the C3/C5
# rocprof summaries.  usage: tools/r3_final.sh OUT
OUT=${1:-gpurun_out/r3_final}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { cat "$OUT/smoke.txt"; exit 1; }
cat "$OUT/smoke.txt"
bash tools/r3_benches.sh "$OUT/bench" || exit 1
timeout -k 10 300 python tools/shard_probe.py 8 > "$OUT/shards8.txt" 2>&1 || exit 1
tail -1 "$OUT/shards8.txt"
