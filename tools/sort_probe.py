"""Does ray order matter for traversal?  Traces the same secondary extension
rays (oracle-recorded, 1280x720 frame 3) in path order, shuffled, and sorted by
(direction octant, Morton code of the origin); run under rocprofv3 --kernel-trace."""
import sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import numpy as np
import torch  # noqa: F401
import surf_amd

def morton(o, lo, hi, bits=8):
    q = np.clip(((o - lo) / (hi - lo) * (1 << bits)).astype(np.int64), 0, (1 << bits) - 1)
    code = np.zeros(len(o), np.int64)
    for b in range(bits):
        for a in range(3):
            code |= ((q[:, a] >> b) & 1) << (3 * b + a)
    return code

z = np.load("/root/repo/gpurun_in_rays.npz")
o, d = z["eo"], z["ed"]
so, sd, st = z["so"], z["sd"], z["st"]
lo, hi = o.min(0), o.max(0)
rng = np.random.default_rng(0)
orders = {
    "path": np.arange(len(o)),
    "shuffled": rng.permutation(len(o)),
    "oct+morton": np.lexsort((morton(o, lo, hi), ((d[:, 0] > 0) * 4 + (d[:, 1] > 0) * 2 + (d[:, 2] > 0)))),
    "morton+oct": np.lexsort((((d[:, 0] > 0) * 4 + (d[:, 1] > 0) * 2 + (d[:, 2] > 0)), morton(o, lo, hi, 6))),
}
s = surf_amd.Scene.indoor()
r = surf_amd.Renderer(s, 64, 64)
for rep in range(2):
    for name, idx in orders.items():
        print(rep, name, flush=True)
        r.trace_closest(o[idx], d[idx])
sorder = np.lexsort((morton(so, lo, hi), ((sd[:, 0] > 0) * 4 + (sd[:, 1] > 0) * 2 + (sd[:, 2] > 0))))
for rep in range(2):
    r.trace_any(so, sd, st)
    r.trace_any(so[sorder], sd[sorder], st[sorder])
print("done")
