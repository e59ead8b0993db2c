#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-ab_pf}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
bash tools/ab_libs.sh ${1:-ab_pf} default surf-path-tracer_amd/lib/variants/pf0.so
