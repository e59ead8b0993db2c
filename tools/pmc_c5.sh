#!/bin/bash
# PMC passes over one C5 render (k_extend on the 10.2M-triangle BLAS): cache,
# latency, TLB and issue counters, one pass each (MI355X_MICROARCH.md slots).
set -o pipefail
OUT=${1:-gpurun_out/pmc_c5}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
CMD="python3 bench.py --workload C5 --steps 1 --warmup 0 --no-cpu --profile-pass 0"
i=0
for set in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_BUSY_CYCLES" \
           "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_PERMISSION_MISS_sum TCP_UTCL1_REQUEST_sum"; do
  i=$((i+1))
  timeout -s KILL 100 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.json 2> $OUT/p$i.err || echo "pass $i failed: $set"
done
echo done
