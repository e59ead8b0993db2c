"""Summarises a SURF_DRAIN_TRACE_FILE: active paths over time, the longest
paths, and how the state a path enters the drain with (age, inMedium,
lastSpecular, max(T)) predicts its remaining segments (diagnostics)."""
import sys
import numpy as np

for path in sys.argv[1:]:
    rows = [l.split() for l in open(path) if not l.startswith("#")]
    hdr = [l for l in open(path) if l.startswith("#")][0]
    khz = float(hdr.split("clock")[1].split("kHz")[0])
    a = np.array(rows, dtype=np.int64)
    end_lo, state, seg, start_lo = a[:, 0], a[:, 1], a[:, 2].astype(np.float64), a[:, 3]
    ref = start_lo.min()
    s = ((start_lo - ref) % (1 << 32)) / khz
    e = ((end_lo - ref) % (1 << 32)) / khz
    age = state & 0xFFFF
    med = (state >> 16) & 1
    spec = (state >> 17) & 1
    mt = ((state >> 24) & 0xFF) / 255.0
    print(path, f"{len(a)} paths, {seg.sum():.0f} segments, drain {e.max():.1f} ms")
    for q in (0.5, 0.9, 0.99, 0.999, 1.0):
        print(f"  paths done by {np.quantile(e, q):7.2f} ms: {q:.3f}")
    for t in (5, 20, 40, 80, 120, 160, 200, 240):
        alive = ((s <= t) & (e > t)).sum()
        print(f"  t={t:4d} ms: {alive:6d} paths active, {seg[e <= t].sum() / seg.sum():.3f} of segments in finished paths")
    for i in np.argsort(-seg)[:6]:
        print(f"  long path: {seg[i]:.0f} segments, {s[i]:.2f} -> {e[i]:.2f} ms, {(e[i]-s[i])*1e3/seg[i]:.1f} us/segment,"
              f" age {age[i]} medium {med[i]} spec {spec[i]} maxT {mt[i]:.3f}")
    long = seg >= 1000
    print(f"  paths >= 1000 segments: {long.sum()}; medium {med[long].mean():.2f} (all {med.mean():.2f}),"
          f" maxT>=0.99 {(mt[long] >= 0.99).mean():.2f} (all {(mt >= 0.99).mean():.2f}), age median {np.median(age[long])} (all {np.median(age)})")
    for name, m in (("medium", med == 1), ("maxT>=0.99", mt >= 0.99), ("maxT>=0.99|medium", (mt >= 0.99) | (med == 1)),
                     ("age>=64", age >= 64)):
        print(f"  {name:20s}: {m.sum():6d} paths, {seg[m].sum() / seg.sum():.3f} of segments, mean {seg[m].mean() if m.any() else 0:.0f} vs {seg[~m].mean():.0f}")
