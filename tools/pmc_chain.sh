#!/bin/bash
# SQ counters of k_tail_coop on the single-path chain probe (one long path per wave, alone).
set -o pipefail
OUT=${1:-gpurun_out/pmc_chain}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CMD="python3 tools/chain_probe2.py"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  SURF_TAIL_ROWS=0 timeout -s KILL 100 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.txt 2> $OUT/p$i.err || echo "pass $i failed"
done
echo done
