#!/bin/bash
# Cache-hierarchy counters for the wavefront kernels (one group per pass).
set -e
OUT=${1:-gpurun_out/pmc_cache}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CMD="python3 bench.py --steps 1 --warmup 0 --no-cpu --profile-pass 0"
i=0
for grp in "TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES" \
           "TCC_HIT TCC_MISS TCC_REQ" \
           "TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- $CMD > "$OUT/p$i.json" 2> "$OUT/p$i.err"
done
echo done
