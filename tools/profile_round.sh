#!/bin/bash
# Collects the rocprofv3 evidence of one bench workload on the GPU box:
#   trace/  kernel trace + stats of the bench command (graph replays, as timed)
#   fetch/  FETCH_SIZE pass, write/  WRITE_SIZE pass (separate passes: TCC
#           slots, MI355X_MICROARCH.md "rocprofv3 PMC slots")
#   sqa/ sqb/  two SQ passes: instruction mix; issuing / waiting / stalled wave
#           cycles and VALU lane utilization (the issue-side roofline)
# then tools/summarize_profile.py writes OUTDIR/summary.json, the kernel stats
# are kept as OUTDIR/kernel_stats.csv and the raw pass directories removed.
# usage: tools/profile_round.sh OUTDIR [WORKLOAD [STEPS]]
set -e
OUT=${1:-gpurun_out/prof}
WL=${2:-C3}
STEPS=${3:-2}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CMD="bench.py --workload $WL --steps $STEPS --warmup 1 --no-cpu --profile-pass 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 $CMD > "$OUT/bench_traced.json" 2> "$OUT/trace.err"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 $CMD > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 $CMD > "$OUT/bench_write.json" 2> "$OUT/write.err"
# issue side (MI355X_MICROARCH.md "rocprofv3 PMC slots": 8 SQ counters per pass): instruction mix, then
# where the waves' cycles go (issuing / parked on s_waitcnt / issue-stalled) and the VALU lane utilization
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_FLOPS_FP64 \
    --output-format csv -d "$OUT/sqa" -o run -- python3 $CMD > "$OUT/bench_sqa.json" 2> "$OUT/sqa.err"
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM \
    --output-format csv -d "$OUT/sqb" -o run -- python3 $CMD > "$OUT/bench_sqb.json" 2> "$OUT/sqb.err"
python3 tools/summarize_profile.py "$OUT" "$OUT/summary.json" "python3 $CMD" "$WL" > /dev/null
# keep the reductions only: the raw per-dispatch CSVs of five passes exceed what a gpurun call brings back
cp "$OUT/trace/run_kernel_stats.csv" "$OUT/kernel_stats.csv"
rm -rf "$OUT/trace" "$OUT/fetch" "$OUT/write" "$OUT/sqa" "$OUT/sqb"
echo done
