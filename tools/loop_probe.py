"""The drop-in frame loop from Python (main.cpp:381-446 shape): F per-frame
render(1) calls, then one synchronize; prints Mrays/s.  Diagnostics only.
    SURF_HIP_LIB=<variant> python tools/loop_probe.py [F]"""
import json, sys, time
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/surf-path-tracer_amd")
import torch  # noqa: F401
import surf_amd
F = int(sys.argv[1]) if len(sys.argv) > 1 else 256
W, H = 1280, 720
r = surf_amd.Renderer(surf_amd.Scene.indoor(), W, H)
r.render(4, 0, 0); r.synchronize(); r.clear_accumulator()
for rep in range(2):
    r.clear_accumulator()
    t = time.perf_counter()
    for f in range(F):
        r.render(1, 1000 + rep * F + f, 0)
    r.synchronize()
    dt = time.perf_counter() - t
    print(json.dumps({"frames": F, "loop_ms": round(dt * 1e3, 1), "mrays_per_s": round(W * H * F / dt / 1e6, 1)}), flush=True)
