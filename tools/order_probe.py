"""Does ray order matter to the closest-hit kernel?  Extension rays of a
1280x720 frame band (oracle-recorded, every segment of every path) traced by
k_trace_closest in: recorded order, shuffled, sorted by hit instance, sorted
by a key of the BVH instances whose (world) boxes the ray crosses.  Kernel
times from rocprofv3 --kernel-trace.  Diagnostics."""
import sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import numpy as np
import torch  # noqa: F401
import oracle
import surf_amd

os_ = oracle.OracleScene()
(eo, ed), _ = os_.record_rays(1280, 720, 0, 300 * 1280, 420 * 1280, max_ext=1 << 21, max_shadow=1)
print("rays", len(eo), flush=True)
t, inst, prim = os_.trace_closest(eo, ed)[0], os_.trace_closest(eo, ed)[3], None
s = surf_amd.Scene.indoor()
r = surf_amd.Renderer(s, 64, 64)
rng = np.random.default_rng(1)
orders = {"recorded": np.arange(len(eo)), "shuffled": rng.permutation(len(eo)),
          "by_hit_instance": np.argsort(inst, kind="stable")}
# world-space box key: bounding boxes of the BVH instances (from the export) are not exposed;
# approximate with the oracle's per-instance node visits > 1 (the ray entered that BLAS)
nodes, _ = os_.trace_visits(eo, ed)
key = ((nodes > 1).astype(np.uint32) << np.arange(nodes.shape[1], dtype=np.uint32)).sum(1)
orders["by_entered_instances"] = np.argsort(key, kind="stable")
for name, o in orders.items():
    for rep in range(3):
        r.trace_closest(eo[o], ed[o])
    print(name, "done", flush=True)
