"""Does ray order matter to the closest-hit kernel?  Extension rays of a
1280x720 frame band (oracle-recorded, every segment of every path) traced by
k_trace_closest in several orders: recorded (path-major), shuffled, sorted by
the BVH instances each ray enters (expensive to know), and by cheap stable
keys a wavefront kernel could compute (direction octant, coarse origin cell,
the instance the ray starts on).  Kernel times: rocprofv3 --kernel-trace.
Diagnostics."""
import sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import numpy as np
import torch  # noqa: F401
import oracle
import surf_amd

os_ = oracle.OracleScene()
(eo, ed), _ = os_.record_rays(1280, 720, 0, 300 * 1280, 420 * 1280, max_ext=1 << 21, max_shadow=1)
print("rays", len(eo), flush=True)
_, _, _, inst, _ = os_.trace_closest(eo, ed)
nodes, _ = os_.trace_visits(eo, ed)
rng = np.random.default_rng(1)
shuf = rng.permutation(len(eo))
eo, ed, inst, nodes = eo[shuf], ed[shuf], inst[shuf], nodes[shuf]      # start from a shuffled pool
# the instance each ray starts on: the closest hit of a short ray backwards from its origin
_, _, _, start, _ = os_.trace_closest(eo + 1e-3 * ed, -ed)
start = np.where(start == 0xFFFFFFFF, 15, start).astype(np.uint32)
octant = ((ed[:, 0] < 0).astype(np.uint32) | ((ed[:, 1] < 0).astype(np.uint32) << 1) | ((ed[:, 2] < 0).astype(np.uint32) << 2))
lo, hi = eo.min(0), eo.max(0)
cell = np.clip(((eo - lo) / (hi - lo + 1e-9) * 4).astype(np.uint32), 0, 3)
cellk = cell[:, 0] | (cell[:, 1] << 2) | (cell[:, 2] << 4)
entered = ((nodes > 1).astype(np.uint32) << np.arange(nodes.shape[1], dtype=np.uint32)).sum(1)
keys = {"shuffled": np.zeros(len(eo), np.uint32), "entered_instances": entered, "octant": octant,
        "start_instance": start, "start+octant": start * 8 + octant, "cell+octant": cellk * 8 + octant,
        "start+cell+octant": (start * 64 + cellk) * 8 + octant}
s = surf_amd.Scene.indoor()
r = surf_amd.Renderer(s, 64, 64)
for name, k in keys.items():
    o = np.argsort(k, kind="stable")
    for rep in range(3):
        r.trace_closest(eo[o], ed[o])
    print(name, flush=True)
