#!/bin/bash
# One GPU-box session: -m gpu tests, the default bench line, the rocprofv3
# evidence of the C3 workload.  usage: tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-r2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
bash tools/profile_round.sh "$OUT/prof" C3 2 || { echo "profile failed"; exit 1; }
echo ok
