#!/bin/bash
# Collects the rocprofv3 evidence for one round on the GPU box:
#   trace/  kernel trace + stats of the bench command
#   fetch/  FETCH_SIZE pass, write/  WRITE_SIZE pass (separate passes:
#           TCC slots, MI355X_MICROARCH.md "rocprofv3 PMC slots")
# usage: tools/profile_round.sh OUTDIR [STEPS]
set -e
OUT=${1:-gpurun_out/prof}
STEPS=${2:-16}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --steps "$STEPS" --warmup 1 --no-cpu > "$OUT/bench_traced.json" 2> "$OUT/trace.err"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 bench.py --steps "$STEPS" --warmup 1 --no-cpu --profile-pass 0 > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 bench.py --steps "$STEPS" --warmup 1 --no-cpu --profile-pass 0 > "$OUT/bench_write.json" 2> "$OUT/write.err"
echo done
