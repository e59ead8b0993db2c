"""Closest-hit latency of the red Suzanne's interior rays in the lane traversal
(k_trace_closest, one ray per lane) and the cooperative one (k_trace_closest_coop,
one ray per wave), on batches of the long C3 path's extension rays
(tools/chainpath_rays.npz): under rocprofv3 --kernel-trace the kernel durations
give how long a small batch of such rays keeps each traversal busy -- the floor
of a small wavefront phase.  Diagnostics only.
    python tools/lane_vs_coop.py"""
import os
import sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import numpy as np
import torch  # noqa: F401
import surf_amd

z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "chainpath_rays.npz"))
scene = surf_amd.Scene.indoor()
r = surf_amd.Renderer(scene, 1280, 720)
eo, ed = z["eo"].astype(np.float32), z["ed"].astype(np.float32)
for mode in (0, 1):
    r.set_trace_mode(mode)
    for n in (1, 64, 512, 3086):
        for rep in range(3):
            t, u, v, inst, prim = r.trace_closest(eo[:n], ed[:n])
        print("mode", mode, "rays", n, "hits", int((inst != 0xffffffff).sum()), flush=True)
