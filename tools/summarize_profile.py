"""Summarizes a tools/profile_round.sh output directory into a small JSON
(kernel durations + HBM traffic per k_extend launch) for profiles/.

FETCH_SIZE / WRITE_SIZE are in KiB.  gfx950 correction (MI355X_MICROARCH.md
§HBM): FETCH_SIZE counts half the bytes of a wide (16 B/lane) coalesced read,
so the read side is doubled; WRITE_SIZE is exact for 16-B stores.  The
traversal's node/triangle fetches are 16-B vector loads too.
usage: python tools/summarize_profile.py DIR OUT.json [COMMAND [WORKLOAD]]
"""
import csv
import json
import statistics
import sys


def short(name):
    return name.split("(")[0].split("::")[-1]


def kernel_stats(path):
    out = {}
    for r in csv.DictReader(open(path)):
        out[short(r["Name"])] = {"calls": int(r["Calls"]), "total_ms": int(r["TotalDurationNs"]) / 1e6,
                                 "avg_us": float(r["AverageNs"]) / 1e3, "pct": float(r["Percentage"])}
    return out


def counter(path, kernel, name):
    """Per-dispatch values of one counter for kernels whose short name starts with `kernel`."""
    per = {}
    for r in csv.DictReader(open(path)):
        if short(r["Kernel_Name"]).startswith(kernel) and r["Counter_Name"] == name:
            per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(per.values())


def counter_by_kernel(path, name):
    """{kernel short name: per-dispatch values} of one counter."""
    per = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name:
            k = short(r["Kernel_Name"])
            per.setdefault(k, {})
            per[k][r["Dispatch_Id"]] = per[k].get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return {k: list(v.values()) for k, v in per.items()}


# Issue-side roofline (VERDICT r5 "What's weak" #4): a traversal kernel is bound by
# dependent loads and divergent / scalar issue, not by HBM bytes, so the bench
# line also reports where its waves' cycles go.  Peak VALU issue: one wave64 VALU
# instruction per 2 cycles per SIMD (SIMD-32, MI355X_MICROARCH.md cycle
# constants), 1024 SIMDs at the 2.4 GHz peak engine clock.
SIMDS, CLOCK_HZ = 1024, 2.4e9
VALU_PEAK = SIMDS * CLOCK_HZ / 2.0          # wave-instructions per second
SQ_A = ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH",
        "SQ_INSTS_VALU_FLOPS_FP64")
SQ_B = ("SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_THREAD_CYCLES_VALU",
        "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_VMEM")


def issue_block(d, ks, bench, kernel, unit_name, units_per_launch):
    """Per-unit instruction mix and cycle split of `kernel` from the SQ passes."""
    import os
    fa, fb = f"{d}/sqa/run_counter_collection.csv", f"{d}/sqb/run_counter_collection.csv"
    if not (os.path.exists(fa) and os.path.exists(fb)) or not units_per_launch:
        return None
    tot = {}
    launches = 0
    for path, names in ((fa, SQ_A), (fb, SQ_B)):
        for n in names:
            v = counter(path, kernel, n)
            if v:
                tot[n] = sum(v)
                launches = max(launches, len(v))
    if not launches or "SQ_INSTS_VALU" not in tot:
        return None
    units = units_per_launch * launches
    per = lambda n: round(tot[n] / units, 2) if n in tot else None
    k = next((v for n, v in ks.items() if n.startswith(kernel)), None)
    avg_s = k["avg_us"] * 1e-6 if k else None
    wc = tot.get("SQ_WAVE_CYCLES")
    blk = {"kernel": kernel, "unit": unit_name, "units_per_launch": round(units_per_launch, 1), "launches": launches,
           "per_unit": {"valu": per("SQ_INSTS_VALU"), "salu": per("SQ_INSTS_SALU"), "vmem_rd": per("SQ_INSTS_VMEM_RD"),
                        "smem": per("SQ_INSTS_SMEM"), "lds": per("SQ_INSTS_LDS"), "branch": per("SQ_INSTS_BRANCH"),
                        "valu_fp64": per("SQ_INSTS_VALU_FLOPS_FP64")},
           "wave_cycles_split": {"issuing": round(tot["SQ_ACTIVE_INST_ANY"] / wc, 4) if wc and "SQ_ACTIVE_INST_ANY" in tot else None,
                                 "waitcnt": round(tot["SQ_WAIT_ANY"] / wc, 4) if wc and "SQ_WAIT_ANY" in tot else None,
                                 "issue_stall": round(tot["SQ_WAIT_INST_ANY"] / wc, 4) if wc and "SQ_WAIT_INST_ANY" in tot else None},
           "valu_lane_utilization": round(tot["SQ_THREAD_CYCLES_VALU"] / (64.0 * tot["SQ_ACTIVE_INST_VALU"]), 4)
                                    if tot.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in tot else None}
    if avg_s:
        achieved = tot["SQ_INSTS_VALU"] / launches / avg_s
        blk["valu_issue"] = {"achieved": round(achieved / 1e9, 3), "peak": round(VALU_PEAK / 1e9, 1), "unit": "G wave-instr/s",
                             "frac": round(achieved / VALU_PEAK, 4)}
    split = blk["wave_cycles_split"]
    if split["waitcnt"] is not None:
        blk["binding"] = ("memory latency (waves parked on s_waitcnt)" if split["waitcnt"] >= max(split["issuing"], split["issue_stall"])
                          else "instruction issue" if split["issuing"] >= split["issue_stall"] else "issue dependencies / pipe stalls")
    return blk


def main():
    d, out = sys.argv[1], sys.argv[2]
    cmd = sys.argv[3] if len(sys.argv) > 3 else "python3 bench.py --steps 16 --warmup 1 --no-cpu"
    workload = sys.argv[4] if len(sys.argv) > 4 else "C3"
    ks = kernel_stats(f"{d}/trace/run_kernel_stats.csv")
    fetch = counter(f"{d}/fetch/run_counter_collection.csv", "k_extend", "FETCH_SIZE")
    write = counter(f"{d}/write/run_counter_collection.csv", "k_extend", "WRITE_SIZE")
    bench = json.loads(open(f"{d}/bench_traced.json").read().strip().splitlines()[-1])
    fk = counter_by_kernel(f"{d}/fetch/run_counter_collection.csv", "FETCH_SIZE")
    wk = counter_by_kernel(f"{d}/write/run_counter_collection.csv", "WRITE_SIZE")
    by_kernel = {}
    for k in sorted(set(fk) | set(wk)):
        f, w = fk.get(k, []), wk.get(k, [])
        by_kernel[k] = {"launches": len(f), "fetch_kib_avg_raw": statistics.mean(f) if f else None,
                        "write_kib_avg": statistics.mean(w) if w else None,
                        "hbm_bytes_per_launch_corrected": (2 * statistics.mean(f) + statistics.mean(w)) * 1024 if f and w else None}
    res = {
        "command": cmd + "  (under rocprofv3 --kernel-trace --stats; PMC passes: the same command, one counter per pass)",
        "workload": workload,
        "kernels": ks,
        "bench_value_traced": bench["value"],
        "k_extend_pmc": {
            "launches": len(fetch),
            "fetch_kib_avg_raw": statistics.mean(fetch) if fetch else None,
            "write_kib_avg": statistics.mean(write) if write else None,
            "hbm_bytes_per_launch_corrected": (2 * statistics.mean(fetch) + statistics.mean(write)) * 1024 if fetch and write else None,
            "correction": "read side x2 (gfx950 FETCH_SIZE halves 16-B/lane reads), KiB x1024",
        },
        "pmc_by_kernel": by_kernel,
    }
    # units: bench.py's events of its last render (every render of the command has the same workload)
    epr = bench.get("events_per_render") or {}
    iters = epr.get("iterations") or 0
    issue = {}
    if iters and epr.get("n_ext_wavefront"):
        issue["k_extend"] = issue_block(d, ks, bench, "k_extend", "extension ray traced by k_extend", epr["n_ext_wavefront"] / iters)
    if iters and epr.get("n_ext_wavefront"):
        issue["k_shade"] = issue_block(d, ks, bench, "k_shade", "pool path shaded by k_shade", epr["n_ext_wavefront"] / iters)
    if iters and epr.get("n_shadow") and epr.get("n_ext"):
        # the wavefront phases' shadow rays, estimated as the wavefront share of the extension rays
        issue["k_connect"] = issue_block(d, ks, bench, "k_connect", "shadow ray traced by k_connect (wavefront share, estimated)",
                                         epr["n_shadow"] * epr["n_ext_wavefront"] / epr["n_ext"] / iters)
    if epr.get("drain_segments"):
        issue["k_tail_pair"] = issue_block(d, ks, bench, "k_tail_pair", "drain segment (extension ray of the drain)",
                                           epr["drain_segments"])
    res["issue"] = {k: v for k, v in issue.items() if v}
    # every kernel's SQ counter totals over the command (the raw passes are not committed)
    import os
    sq = {}
    for path, names in ((f"{d}/sqa/run_counter_collection.csv", SQ_A), (f"{d}/sqb/run_counter_collection.csv", SQ_B)):
        if not os.path.exists(path):
            continue
        for n in names:
            for k, v in counter_by_kernel(path, n).items():
                sq.setdefault(k, {"launches": len(v)})[n] = sum(v)
    if sq:
        res["sq_totals_by_kernel"] = sq
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
