#!/bin/bash
# Per-kernel PMC attribution over bench variants (one C3-class render per pass):
#   tools/pmc_variants.sh OUT KERNEL 'PASS;PASS;...' 'name|ENV=V,ENV=V|--bench-opts' ...
# Each PASS is one rocprofv3 --pmc run (counters separated by spaces, within the
# per-block limits of MI355X_MICROARCH.md); the summary prints, per variant and
# pass, the mean per launch of every counter over the launches of KERNEL
# (substring match), and the bench line's profile-pass kernel times.
OUT=${1:?out dir}; KERN=${2:?kernel}; PASSES=${3:?passes}; shift 3
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
IFS=';' read -r -a PL <<< "$PASSES"
for v in "$@"; do
  IFS='|' read -r name envs opts <<< "$v"
  k=0
  for pass in "${PL[@]}"; do
    ( IFS=,; for e in $envs; do [ -n "$e" ] && export "$e"; done; unset IFS
      timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d "$OUT/${name}_p$k" -o run -- \
        python3 bench.py --steps 1 --warmup 0 --no-cpu $opts > "$OUT/${name}_p$k.json" 2> "$OUT/${name}_p$k.err" ) || exit 1
    k=$((k + 1))
  done
done
python3 - "$OUT" "$KERN" "${#PL[@]}" "$@" <<'PY'
import csv, glob, json, statistics, sys
out, kern, npass = sys.argv[1], sys.argv[2], int(sys.argv[3])
for v in sys.argv[4:]:
    name = v.split("|")[0]
    res = {"variant": name}
    for k in range(npass):
        files = glob.glob(f"{out}/{name}_p{k}/**/run_counter_collection.csv", recursive=True) + \
            glob.glob(f"{out}/{name}_p{k}/run_counter_collection.csv")
        per = {}
        for f in set(files):
            for r in csv.DictReader(open(f)):
                if kern in r["Kernel_Name"]:
                    per.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        for c, vals in per.items():
            res[c] = statistics.mean(vals)
            res["launches"] = len(vals)
        try:
            j = json.load(open(f"{out}/{name}_p{k}.json"))
            res["value"] = j["value"]
            res["kernel_ms"] = j.get("kernel_ms_profile_pass")
        except Exception:
            pass
    if "FETCH_SIZE" in res:
        res["fetch_corrected_MB"] = round(2 * res["FETCH_SIZE"] * 1024 / 1e6, 1)
    if "WRITE_SIZE" in res:
        res["write_MB"] = round(res["WRITE_SIZE"] * 1024 / 1e6, 1)
    if "TCC_HIT_sum" in res and "TCC_MISS_sum" in res:
        res["l2_hit"] = round(res["TCC_HIT_sum"] / max(1.0, res["TCC_HIT_sum"] + res["TCC_MISS_sum"]), 4)
    print(json.dumps(res))
PY
