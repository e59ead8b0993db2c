"""Control vs memory divergence: distinct rays ordered so that each wave's rays
take the same number of node visits per instance (trip-count coherent, memory
divergent) vs random order.  Run under rocprofv3 --kernel-trace."""
import sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import numpy as np
import torch  # noqa: F401
import surf_amd
import oracle
z = np.load("/root/repo/gpurun_in_rays.npz")
o, d = z["eo"][:500000], z["ed"][:500000]
osc = oracle.OracleScene()
nodes, tris = osc.trace_visits(o, d)
keys = np.concatenate([nodes, tris], axis=1)
order = np.lexsort(keys.T[::-1])
rng = np.random.default_rng(0)
shuf = rng.permutation(len(o))
s = surf_amd.Scene.indoor()
r = surf_amd.Renderer(s, 64, 64)
for k in range(2):
    r.trace_closest(o[shuf], d[shuf])
    r.trace_closest(o[order], d[order])
print("done")
