"""Where a drain segment's latency goes (diagnostics): surf_debug_segment_cycles
on extension rays of the long C3 path of tools/chain_probe.py (pixel 630758,
frame 0: 3086 segments inside the red Suzanne; rays recorded once from the
oracle into tools/chainpath_rays.npz), one lone wave, each piece repeated.
    python tools/segment_cycles.py [N_RAYS]"""
import json
import os
import sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import numpy as np
import torch  # noqa: F401
import surf_amd

n = int(sys.argv[1]) if len(sys.argv) > 1 else 48
z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "chainpath_rays.npz"))
scene = surf_amd.Scene.indoor()
r = surf_amd.Renderer(scene, 1280, 720)
acc = {}
rng = np.random.default_rng(3)
idx = np.linspace(50, len(z["eo"]) - 50, n).astype(int)
for k in idx:
    c = r.debug_segment_cycles(z["eo"][k], z["ed"][k], (1.0, 0.0, 0.0), int(rng.integers(1, 2**32 - 1)), segment=100, reps=32)
    for key, v in c.items():
        acc.setdefault(key, []).append(v)
out = {k: round(float(np.mean(v)), 1) for k, v in acc.items()}
out["rays"] = int(n)
out["lib"] = os.environ.get("SURF_HIP_LIB", "default")
print(json.dumps(out))
