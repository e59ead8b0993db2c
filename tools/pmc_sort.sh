#!/bin/bash
# k_extend HBM-side traffic with and without the ray-order gather (SURF_SORT=1 vs 0):
# FETCH_SIZE and WRITE_SIZE in separate passes (TCC slots), one C3 render each.
# usage: tools/pmc_sort.sh OUTDIR
set -e
OUT=${1:-gpurun_out/pmc_sort}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for s in 1 0; do
  for c in FETCH_SIZE WRITE_SIZE; do
    SURF_SORT=$s timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$OUT/s${s}_$c" -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu --profile-pass 0 > "$OUT/s${s}_$c.json" 2> "$OUT/s${s}_$c.err"
  done
done
python3 - "$OUT" <<'PY'
import csv, json, statistics, sys
out = sys.argv[1]
for s in (1, 0):
    v = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = [r for r in csv.DictReader(open(f"{out}/s{s}_{c}/run_counter_collection.csv"))
                if "k_extend" in r["Kernel_Name"] and r["Counter_Name"] == c]
        v[c] = statistics.mean(float(r["Counter_Value"]) for r in rows) * 1024
        v["launches"] = len(rows)
    b = json.load(open(f"{out}/s{s}_FETCH_SIZE.json"))
    print(json.dumps({"sort": s, "launches": v["launches"], "fetch_raw_MB": round(v["FETCH_SIZE"] / 1e6, 1),
                      "write_MB": round(v["WRITE_SIZE"] / 1e6, 1),
                      "corrected_MB": round((2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) / 1e6, 1), "value": b["value"]}))
PY
