#!/bin/bash
# Occupancy / in-flight PMC passes over tools/c5_probe.py.
set -e
OUT=gpurun_out/pmc_c5b
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for set in "SQ_LEVEL_WAVES GRBM_GUI_ACTIVE SQ_WAVES SQ_CYCLES" \
           "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS" \
           "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 tools/c5_probe.py > $OUT/p$i.log 2>&1
done
echo done
