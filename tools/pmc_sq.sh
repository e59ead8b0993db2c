#!/bin/bash
# SQ counter passes (issue vs latency diagnosis) for the wavefront kernels.
set -e
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CMD="python3 bench.py --steps 1 --warmup 0 --no-cpu --profile-pass 0"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_BRANCH \
    --output-format csv -d "$OUT/a" -o run -- $CMD > "$OUT/a.json" 2> "$OUT/a.err"
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_LEVEL_WAVES \
    --output-format csv -d "$OUT/b" -o run -- $CMD > "$OUT/b.json" 2> "$OUT/b.err"
echo done
