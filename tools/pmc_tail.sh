#!/bin/bash
# SQ counters (issue vs latency) of the drain kernels, both engines, one C3 render each.
set -e
OUT=${1:-gpurun_out/pmc_tail}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CMD="python3 bench.py --steps 1 --warmup 0 --no-cpu --profile-pass 0"
for m in 0 1; do
SURF_TAIL_ROWS=$m timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES \
    --output-format csv -d "$OUT/a$m" -o run -- $CMD > "$OUT/a$m.json" 2> "$OUT/a$m.err"
SURF_TAIL_ROWS=$m timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LEVEL_WAVES \
    --output-format csv -d "$OUT/b$m" -o run -- $CMD > "$OUT/b$m.json" 2> "$OUT/b$m.err"
done
echo done
