#!/bin/bash
set -e
OUT=gpurun_out/pmc_div
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/a -o run -- python3 tools/divergence_probe.py > $OUT/a.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ --output-format csv -d $OUT/b -o run -- python3 tools/divergence_probe.py > $OUT/b.log 2>&1
echo done
