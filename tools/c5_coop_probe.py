"""C5 extension rays (the oracle's record of rows 340..351 of frame 7) traced
one per lane (k_trace_closest) and one per wave (k_trace_closest_coop, the
drain's two-level lanes-as-planes walk): under rocprofv3 --kernel-trace the
two kernels' durations give each traversal's throughput on the HBM-resident
BVH; the hit records must agree.  Diagnostics only.
    python tools/c5_coop_probe.py"""
import os
import sys
import time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "surf-path-tracer_amd"))
import numpy as np
import torch  # noqa: F401
import oracle as O
import surf_amd

O.load()
t = time.time()
S = O.OracleScene(variant=1)
W = 1280
(eo, ed), _ = S.record_rays(W, 720, 7, 340 * W, 352 * W, max_ext=1 << 21, max_shadow=1 << 20)
eo, ed = np.ascontiguousarray(eo, np.float32), np.ascontiguousarray(ed, np.float32)
print("rays", len(eo), "recorded in", round(time.time() - t, 1), "s", flush=True)
p = surf_amd.Scene.indoor(variant=1)
r = surf_amd.Renderer(p, W, 720)
res = {}
for mode in (0, 1):
    r.set_trace_mode(mode)
    for rep in range(3):
        res[mode] = r.trace_closest(eo, ed)
    print("mode", mode, "hits", int((res[mode][3] != 0xffffffff).sum()), flush=True)
same = all(np.array_equal(a.view(np.uint32), b.view(np.uint32)) for a, b in zip(res[0], res[1]))
print("lane == wave hit records:", same, flush=True)
