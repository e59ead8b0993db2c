"""Single-ray traversal latency: k_trace_closest on rays of one long lens path
(tools/longpath_rays.npz, recorded with the oracle, cutoff on, frame 75 pixel
445066).  Run under rocprofv3 --kernel-trace; kernel durations per call size."""
import sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import numpy as np
import torch  # noqa: F401
import surf_amd
z = np.load("/root/repo/tools/longpath_rays.npz")
o, d = z["o"], z["d"]
s = surf_amd.Scene.indoor()
r = surf_amd.Renderer(s, 64, 64)
for mode in (0, 1):
  r.set_trace_mode(mode)
  for rep in range(3):
    for k in (100, 1000, 2000):              # single rays deep in a long path
        r.trace_closest(o[k:k + 1], d[k:k + 1])
    r.trace_closest(o[1000:1064], d[1000:1064])   # 64 rays
    r.trace_closest(o, d)                          # the whole path as a batch
print("done", len(o))
