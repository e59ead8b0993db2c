"""Ray order, second round (diagnostics): extension rays sorted by the start
instance combined with coarse origin cells, and shadow rays sorted by the
light they aim at combined with origin cells.  Same recorded rays as
tools/order_probe.py (1280x720 rows 300..419, frame 0); kernel times from
rocprofv3 --kernel-trace, three launches per key, in the order printed."""
import sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import numpy as np
import torch  # noqa: F401
import oracle
import surf_amd

os_ = oracle.OracleScene()
(eo, ed), (so, sd, st) = os_.record_rays(1280, 720, 0, 300 * 1280, 420 * 1280, max_ext=1 << 21, max_shadow=1 << 21)
print("rays", len(eo), "shadow", len(so), flush=True)
rng = np.random.default_rng(1)
p = rng.permutation(len(eo))
eo, ed = eo[p], ed[p]
q = rng.permutation(len(so))
so, sd, st = so[q], sd[q], st[q]
_, _, _, start, _ = os_.trace_closest(eo + 1e-3 * ed, -ed)
start = np.where(start == 0xFFFFFFFF, 15, start).astype(np.uint32)
# the light a shadow ray aims at: the instance its unbounded ray hits first beyond the segment
_, _, _, light, _ = os_.trace_closest(so + st[:, None] * 0.999 * sd, sd)
light = np.where(light == 0xFFFFFFFF, 15, light).astype(np.uint32)
lo = np.minimum(eo.min(0), so.min(0)); hi = np.maximum(eo.max(0), so.max(0))


def cells(o, n):
    c = np.clip(((o - lo) / (hi - lo + 1e-9) * n).astype(np.uint32), 0, n - 1)
    return c[:, 0] + n * (c[:, 1] + n * c[:, 2])


def cellxz(o, n):
    c = np.clip(((o - lo) / (hi - lo + 1e-9) * n).astype(np.uint32), 0, n - 1)
    return c[:, 0] + n * c[:, 2]


ext = {"start": start, "start+cell2": start * 8 + cells(eo, 2), "start+cellxz2": start * 4 + cellxz(eo, 2),
       "start+cellxz4": start * 16 + cellxz(eo, 4), "start+cell4": start * 64 + cells(eo, 4)}
sh = {"shuffled": np.zeros(len(so), np.uint32), "light": light, "light+cell2": light * 8 + cells(so, 2),
      "light+cell4": light * 64 + cells(so, 4), "light+cellxz4": light * 16 + cellxz(so, 4), "cell4": cells(so, 4)}
s = surf_amd.Scene.indoor()
r = surf_amd.Renderer(s, 64, 64)
for name, k in ext.items():
    o = np.argsort(k, kind="stable")
    for rep in range(3):
        r.trace_closest(eo[o], ed[o])
    print("ext", name, len(np.unique(k)), flush=True)
for name, k in sh.items():
    o = np.argsort(k, kind="stable")
    for rep in range(3):
        r.trace_any(so[o], sd[o], st[o])
    print("shadow", name, len(np.unique(k)), flush=True)
