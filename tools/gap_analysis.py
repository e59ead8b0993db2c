"""Idle time of a rocprofv3 kernel trace (diagnostics): wall span vs the union
of kernel intervals, and the gaps between consecutive kernels grouped by the
(previous, next) kernel pair.
usage: python tools/gap_analysis.py run_kernel_trace.csv [t0_frac t1_frac]
"""
import collections
import csv
import sys


def short(name):
    return name.split("(")[0].split("::")[-1]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    if len(sys.argv) > 3:
        a, b = float(sys.argv[2]), float(sys.argv[3])
        t0, t1 = iv[0][0], iv[-1][1]
        lo, hi = t0 + a * (t1 - t0), t0 + b * (t1 - t0)
        iv = [x for x in iv if lo <= x[0] <= hi]
    per = collections.defaultdict(lambda: [0, 0])
    for s, e, n in iv:
        per[n][0] += 1
        per[n][1] += e - s
    busy, gaps = 0, []
    cs, ce, prev = iv[0][0], iv[0][1], iv[0][2]
    for s, e, n in iv[1:]:
        if s > ce:
            busy += ce - cs
            gaps.append((s - ce, prev, n))
            cs, ce = s, e
        else:
            ce = max(ce, e)
        prev = n
    busy += ce - cs
    span = iv[-1][1] - iv[0][0]
    print(f"kernels {len(iv)}  span {span / 1e6:.2f} ms  busy(union) {busy / 1e6:.2f} ms  idle {(span - busy) / 1e6:.2f} ms")
    for n, (c, t) in sorted(per.items(), key=lambda x: -x[1][1]):
        print(f"  {n:28s} calls {c:6d}  total {t / 1e6:9.2f} ms  avg {t / c / 1e3:9.1f} us")
    agg = collections.defaultdict(lambda: [0, 0])
    for g, a, b in gaps:
        agg[(a, b)][0] += 1
        agg[(a, b)][1] += g
    print("gaps by (previous -> next):")
    for (a, b), (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:12]:
        print(f"  {a:22s} -> {b:22s} n {c:6d}  total {t / 1e6:8.2f} ms  avg {t / c / 1e3:8.1f} us")


if __name__ == "__main__":
    main()
