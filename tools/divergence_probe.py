"""Upper bound on what lane coherence could buy: traversal time of 1.5 M
identical rays vs 1.5 M distinct secondary rays (same average work per ray
when a median-cost ray is replicated).  Run under rocprofv3 --kernel-trace."""
import sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import numpy as np
import torch  # noqa: F401
import surf_amd
import oracle
z = np.load("/root/repo/gpurun_in_rays.npz")
o, d = z["eo"], z["ed"]
osc = oracle.OracleScene()
nodes, tris = osc.trace_visits(o[:20000], d[:20000])
cost = nodes.sum(1) * 60 + tris.sum(1) * 55
med = int(np.argsort(cost)[len(cost) // 2])
print("mean nodes/tris", nodes.sum(1).mean(), tris.sum(1).mean(), "median ray", nodes[med].sum(), tris[med].sum())
# a set of ~64 distinct median-ish rays repeated: each wave coherent
sel = np.argsort(np.abs(cost - cost[med]))[:64]
s = surf_amd.Scene.indoor()
r = surf_amd.Renderer(s, 64, 64)
N = len(o)
rep_one = np.repeat(sel[:1], N)
rep_wave = np.tile(np.repeat(sel, 64), N // (64 * 64) + 1)[:N]
for k in range(2):
    r.trace_closest(o, d)                     # distinct
    r.trace_closest(o[rep_one], d[rep_one])   # one median ray everywhere
    r.trace_closest(o[rep_wave], d[rep_wave]) # each wave: one median-ish ray
print("done")
