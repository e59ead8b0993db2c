#!/bin/bash
# Address/data-path counters of the lane traversal kernels (WL=C3 default, C5): is k_extend
# bound by the texture-address unit / L1 (one 16-B access per lane per load)?
# One rocprofv3 --pmc pass per line (block limits: 2 TA, 4 TCP, 2 GRBM).
set -o pipefail
OUT=${1:-gpurun_out/pmc_ta}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CMD="bench.py --workload ${WL:-C3} --steps 1 --warmup 0 --no-cpu --profile-pass 0"
i=0
for pass in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
            "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum" \
            "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_LATENCY_sum" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL ${PASS_TIMEOUT:-120} rocprofv3 --pmc $pass --kernel-include-regex "k_extend|k_connect" --output-format csv -d "$OUT/p$i" -o run -- \
      python3 $CMD > "$OUT/p$i.json" 2> "$OUT/p$i.err" || { echo "pass $i failed"; tail -5 "$OUT/p$i.err"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for i in (1, 2, 3, 4):
    f = glob.glob(f"{out}/p{i}/**/*counter_collection.csv", recursive=True)
    if not f: print("pass", i, "no csv"); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void surfdev::", "").replace("surfdev::", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
    for k, d in acc.items():
        print(i, k, {c: f"{v / n[(k, c)]:.4g}" for c, v in d.items()})
PY
