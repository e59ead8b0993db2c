"""C5 traversal: is a launch bounded by its slowest rays?  Times (rocprofv3
--kernel-trace) k_trace_closest over C5 extension rays: all of them, all but
the 1% / 0.1% most expensive (oracle node-visit counts), and only those.
Input: gpurun_in_c5.npz from `python tools/c5_probe.py --make` (CPU)."""
import sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import numpy as np

VARIANT = 0 if "--indoor" in sys.argv else 1
if "--make" in sys.argv:
    import oracle
    s = oracle.OracleScene(variant=VARIANT)
    (eo, ed), _ = s.record_rays(1280, 720, 0, 0, 1280 * 720 // (8 if VARIANT else 2), max_ext=1_500_000, max_shadow=10)
    n, t = s.trace_visits(eo, ed)
    cost = n.sum(1).astype(np.int64)
    np.savez("/root/repo/gpurun_in_c5.npz", o=eo, d=ed, cost=cost)
    print(len(eo), "rays; nodes/ray mean", cost.mean(), "p99", np.percentile(cost, 99), "p99.9", np.percentile(cost, 99.9), "max", cost.max())
    sys.exit(0)

import torch  # noqa: F401
import surf_amd
z = np.load("/root/repo/gpurun_in_c5.npz")
o, d, cost = z["o"], z["d"], z["cost"]
order = np.argsort(cost)
n = len(o)
sets = {"all": np.arange(n), "drop1%": np.sort(order[: int(n * 0.99)]), "drop0.1%": np.sort(order[: int(n * 0.999)]),
        "top1%": np.sort(order[int(n * 0.99):]), "half": np.arange(n // 2), "quarter": np.arange(n // 4),
        "sixteenth": np.arange(n // 16), "by-cost": order, "shuffled": np.random.default_rng(1).permutation(n),
        "by-dir-octant+origin": np.lexsort((np.round(o[:, 0] * 2), np.round(o[:, 1] * 2), np.round(o[:, 2] * 2), (d > 0) @ np.array([1, 2, 4])))}
s = surf_amd.Scene.indoor(variant=VARIANT)
r = surf_amd.Renderer(s, 64, 64)
import time
for k in range(2):
    for name, idx in sets.items():
        t0 = time.perf_counter()
        r.trace_closest(o[idx], d[idx])
        print(k, name, len(idx), "rays, nodes", int(cost[idx].sum()), f"{(time.perf_counter() - t0) * 1e3:.1f} ms host", flush=True)
