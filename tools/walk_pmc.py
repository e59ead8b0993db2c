"""The closest-hit wave walk alone on a lone wave (surf_debug_segment_cycles with
the walk-only flag), for rocprofv3 --pmc SQ counters of just the walk:
    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU ... -- python tools/walk_pmc.py"""
import os
import sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import numpy as np
import torch  # noqa: F401
import surf_amd
import ctypes as C

z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "chainpath_rays.npz"))
scene = surf_amd.Scene.indoor()
r = surf_amd.Renderer(scene, 1280, 720)
rec = np.zeros(12, np.float32)
out = np.zeros(15, np.uint64)
for k in np.linspace(50, len(z["eo"]) - 50, 16).astype(int):
    rec[0:3] = z["eo"][k]; rec[4:7] = z["ed"][k]; rec[8:11] = (1.0, 0.0, 0.0)
    rc = surf_amd.load().surf_debug_segment_cycles(r._h, rec.ctypes.data, 0x80000000 | 64, out.ctypes.data)
    assert rc == 0
print("walks:", 16 * 64)
